"""Parity of the config workloads (BASELINE.json configs 2-5): device (or the host
emulator of the kernel's step code) vs the oracle -- return bits, trap codes, reference
instruction counts and final-memory hashes, per instance."""
import numpy as np
import pytest

import oracle_py as O
from helpers import compare, emu_run, gpu_run, oracle_run
from wasmedge_amd import workloads as W

I32, I64 = 0x7F, 0x7E

BLAKE3_KATS = {  # test/aot/AOTBlake3Test.cpp:31-77
    b"": "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262",
    b"a": "17762fddd969a453925d65717ac3eea21320b66b54342fde15128d6caf21215f",
    (b"af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262dba5865c"
     b"0d91b17958e4d2cac98c338f85cbbda07b71a020ab16c391b5e7af4b7741362872909e93"
     b"d6ce0779cd18c10aa35222d8b6a8f0bb6c416c69134b73a18409ee61fd95733781993e71"
     b"d9fa298ce39a1150465ed0f2fb995757aefffbca"):
        "e2f3576db165c4c0433fad18533485f7eb00833b33457af59673733505d14f12",
}


def _cases():
    return {
        "blake3": (W.blake3_wasm(), "run", [I32, I32], [I32],
                   [[i, it] for i, it in [(0, 0), (1, 1), (5, 7), (123456, 3), (7, 20)]]),
        "qsort": (W.qsort_wasm(), "sort", [I32, I32], [I32],
                  [[i, n] for i, n in [(0, 0), (1, 1), (2, 2), (3, 17), (4, 500), (99, 2000)]]),
        "collatz": (W.collatz_wasm(), "collatz", [I32, I32], [I32],
                    [[i, 10000] for i in list(range(0, 64)) + [97 * 3, 89 * 2, 83 * 5, 65535]]),
        "mandel": (W.mandel_wasm(), "tile", [I32, I32, I32], [I64],
                   [[i, 128, 50] for i in range(0, 256, 7)]),
    }


def test_blake3_kats_oracle_and_emulator(built):
    for msg, exp in BLAKE3_KATS.items():
        w = W.blake3_kat_wasm(msg)
        m = O.Module(w)
        words = [m.run("kat", [k])[1][0] for k in range(8)]
        assert b"".join(x.to_bytes(4, "little") for x in words).hex() == exp
        rets, st, cnt, h = emu_run(w, "kat", [[k] for k in range(8)], [I32], [I32])
        assert b"".join(r[0].to_bytes(4, "little") for r in rets).hex() == exp


@pytest.mark.parametrize("name", ["blake3", "qsort", "collatz", "mandel"])
def test_workload_emulator_parity(built, name):
    wasm, func, pt, rt, rows = _cases()[name]
    ref = oracle_run(O.Module(wasm), func, rows)
    rets, st, cnt, h = emu_run(wasm, func, rows, pt, rt)
    assert compare(ref, rets, st, cnt, h, rt) == []


@pytest.mark.gpu
def test_gpu_blake3_kats(built):
    for msg, exp in BLAKE3_KATS.items():
        rets, st, cnt, h = gpu_run(W.blake3_kat_wasm(msg), "kat", [[k] for k in range(8)],
                                   [I32], [I32])
        assert b"".join(r[0].to_bytes(4, "little") for r in rets).hex() == exp


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["blake3", "qsort", "collatz", "mandel"])
def test_gpu_workload_parity(built, name):
    wasm, func, pt, rt, rows = _cases()[name]
    ref = oracle_run(O.Module(wasm), func, rows)
    rets, st, cnt, h = gpu_run(wasm, func, rows, pt, rt)
    assert compare(ref, rets, st, cnt, h, rt) == []


@pytest.mark.gpu
def test_gpu_collatz_64k_traps(built):
    """C4 at full size: 64K instances, per-lane traps on ids divisible by 97/89/83."""
    wasm = W.collatz_wasm()
    n = 65536
    rows = [[i, 10000] for i in range(n)]
    rets, st, cnt, h = gpu_run(wasm, "collatz", rows, [I32, I32], [I32])
    m = O.Module(wasm)
    sample = list(range(0, n, 37)) + [97 * 11, 89 * 13, 83 * 17, 0, n - 1]
    ref = oracle_run(m, "collatz", [rows[i] for i in sample])
    sub = lambda a: [a[i] for i in sample]
    assert compare(ref, sub(rets), sub(st), sub(cnt), sub(h), [I32]) == []
    exp_trap = [(0x89 if i % 97 == 0 else 0x84 if i % 89 == 0 else 0x88 if i % 83 == 0 else 0)
                for i in range(n)]
    assert [int(s) for s in st] == exp_trap


@pytest.mark.gpu
def test_gpu_blake3_64k(built):
    """C2 at full width: 64K instances x 20 compressions; every lane vs a sampled oracle
    and the size-independent property that identical ids give identical results."""
    wasm = W.blake3_wasm()
    n = 65536
    rows = [[i % 4096, 20] for i in range(n)]
    rets, st, cnt, h = gpu_run(wasm, "run", rows, [I32, I32], [I32])
    assert all(int(s) == 0 for s in st)
    for i in range(4096, n, 997):
        assert rets[i] == rets[i % 4096] and int(h[i]) == int(h[i % 4096])
    ref = oracle_run(O.Module(wasm), "run", [rows[i] for i in range(0, 4096, 97)])
    idx = list(range(0, 4096, 97))
    assert compare(ref, [rets[i] for i in idx], [st[i] for i in idx], [cnt[i] for i in idx],
                   [h[i] for i in idx], [I32]) == []


@pytest.mark.gpu
@pytest.mark.parametrize("sched", ["0", "1", "4"])
def test_gpu_scheduler_policies_bit_exact(built, sched, monkeypatch):
    """The wave scheduler only decides which lanes run together: min-pc (0) and the
    loop-aware largest-group policy (1, 4) must give identical per-lane results on the
    divergent workloads (quicksort with per-lane data, Collatz with traps)."""
    monkeypatch.setenv("WB_SCHED", sched)
    cases = _cases()
    wasm, func, pt, rt, _ = cases["qsort"]
    cases["qsort"] = (wasm, func, pt, rt, [[i, (i * 37) % 700] for i in range(192)])
    for name in ("qsort", "collatz"):
        wasm, func, pt, rt, rows = cases[name]
        ref = oracle_run(O.Module(wasm), func, rows)
        rets, st, cnt, h = gpu_run(wasm, func, rows, pt, rt)
        assert compare(ref, rets, st, cnt, h, rt) == [], name
