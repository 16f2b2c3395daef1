"""Parity of the config workloads (BASELINE.json configs 2-5): device (or the host
emulator of the kernel's step code) vs the oracle -- return bits, trap codes, reference
instruction counts and final-memory hashes, per instance."""
import os

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
@pytest.mark.parametrize("sched", ["0", "1", "4", "nosimt", "trip", "notrip"])
def test_gpu_scheduler_policies_bit_exact(built, sched, monkeypatch):
    """The wave scheduler only decides which lanes run together: the kernel's min-pc (0)
    and loop-aware largest-group policies (1, 4) between core calls, SIMT scheduling inside
    the compiled runs (default) or not (nosimt: WB_SIMT=0), trip mode forced on or off (WB_TRIP, jit.cpp "Trip
    mode": every lane runs its own compiled run in each trip), must give identical per-lane
    results on the divergent workloads (recursion with per-lane depth, quicksort with
    per-lane data, Collatz's br_table state machine with traps, Mandelbrot's per-lane
    escape)."""
    if sched in ("trip", "notrip"):
        monkeypatch.setenv("WB_TRIP", "1" if sched == "trip" else "0")
    elif sched == "nosimt":
        monkeypatch.setenv("WB_SIMT", "0")
    else:
        monkeypatch.setenv("WB_SCHED", sched)
    cases = _cases()
    wasm, func, pt, rt, _ = cases["qsort"]
    cases["qsort"] = (wasm, func, pt, rt, [[i, (i * 37) % 700] for i in range(192)])
    fib = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fibonacci.wasm"), "rb").read()
    cases["fib"] = (fib, "fib", [I32], [I32], [[(i * 7) % 19] for i in range(192)])
    for name in ("fib", "qsort", "collatz", "mandel"):
        wasm, func, pt, rt, rows = cases[name]
        ref = oracle_run(O.Module(wasm), func, rows)
        rets, st, cnt, h = gpu_run(wasm, func, rows, pt, rt)
        assert compare(ref, rets, st, cnt, h, rt) == [], name


def _oracle_batch(wasm, func, rows, page_limit=65536):
    """The oracle on many instances at once (om_run_batch, host threads), as rows of
    (code, values, count, memhash) for compare()."""
    import os
    m = O.Module(wasm, page_limit=page_limit)
    rows = np.asarray(rows, dtype=np.int64)
    params = np.zeros((len(rows), rows.shape[1], 2), np.uint64)
    params[:, :, 0] = rows.astype(np.uint64)
    out = m.run_batch(func, params, len(rows), threads=min(16, os.cpu_count() or 1))
    res = []
    for i in range(len(rows)):
        code = int(out["codes"][i])
        vals = [int(out["results"][i, 0, 0])] if code == 0 else []
        res.append((code, vals, int(out["counts"][i]), int(out["hashes"][i])))
    return res


def _mask32(rets):
    return [[v[0] & 0xFFFFFFFF] if v else [] for v in rets]


@pytest.mark.gpu
def test_gpu_c2_full_size(built):
    """C2 exactly as configs[1] / bench.py: 64K instances x 1000 chained compressions;
    every 61st instance checked against the oracle, all lanes against each other's
    size-independent property (no traps, identical counts: the loop is data-independent)."""
    wasm = W.blake3_wasm()
    n = 65536
    rows = [[i, 1000] for i in range(n)]
    rets, st, cnt, h = gpu_run(wasm, "run", rows, [I32, I32], [I32])
    assert all(int(s) == 0 for s in st) and len(set(int(c) for c in cnt)) == 1
    idx = list(range(0, n, 61)) + [n - 1]
    ref = _oracle_batch(wasm, "run", [rows[i] for i in idx])
    sub = lambda a: [a[i] for i in idx]
    assert compare(ref, _mask32(sub(rets)), sub(st), sub(cnt), sub(h), [I32]) == []


@pytest.mark.gpu
def test_gpu_c3_64k_x_16k(built):
    """C3 at full width with 16,384 elements per instance (64 KiB of the 1 MiB region):
    a sample of instances bit-exact against the oracle (status, checksum, count, memory
    hash of the sorted region)."""
    wasm = W.qsort_wasm()
    n = 65536
    rows = [[i, 16384] for i in range(n)]
    rets, st, cnt, h = gpu_run(wasm, "sort", rows, [I32, I32], [I32], max_memory_page=17)
    assert all(int(s) == 0 for s in st)
    idx = list(range(0, n, 509)) + [n - 1]
    ref = _oracle_batch(wasm, "sort", [rows[i] for i in idx], page_limit=17)
    sub = lambda a: [a[i] for i in idx]
    assert compare(ref, _mask32(sub(rets)), sub(st), sub(cnt), sub(h), [I32]) == []


@pytest.mark.gpu
def test_gpu_c3_full_size_sample(built):
    """C3 at its configs[2] size, 262,144 i32 (1 MiB) per instance, on one wave of
    instances (ids spread over the 64K range): bit-exact against the oracle. The 64K-wide
    run at this size is bench.py --workload c3 (it checks its CPU-baseline sample too)."""
    wasm = W.qsort_wasm()
    ids = [i * 1021 for i in range(64)]
    rows = [[i, 262144] for i in ids]
    rets, st, cnt, h = gpu_run(wasm, "sort", rows, [I32, I32], [I32], max_memory_page=17)
    ref = _oracle_batch(wasm, "sort", rows, page_limit=17)
    assert compare(ref, _mask32(rets), st, cnt, h, [I32]) == []


@pytest.mark.gpu
def test_gpu_c3_64k_x_1mib(built):
    """C3 exactly as configs[2] / bench.py --workload c3: 64K instances x 262,144 i32
    (64 GiB of linear memory on the device). Every lane must finish without a trap; 48
    instances spread over the batch (both halves of several waves) are bit-exact against
    the oracle (status, checksum, count, memory hash of the whole 17-page memory)."""
    wasm = W.qsort_wasm()
    n = 65536
    rows = [[i, 262144] for i in range(n)]
    rets, st, cnt, h = gpu_run(wasm, "sort", rows, [I32, I32], [I32], max_memory_page=17)
    assert all(int(s) == 0 for s in st)
    assert min(int(c) for c in cnt) > 262144 * 10
    idx = sorted(set([0, 1, 31, 32, 63, 64, n - 1] + list(range(97, n, 1601))))[:48]
    ref = _oracle_batch(wasm, "sort", [rows[i] for i in idx], page_limit=17)
    sub = lambda a: [a[i] for i in idx]
    assert compare(ref, _mask32(sub(rets)), sub(st), sub(cnt), sub(h), [I32]) == []


@pytest.mark.gpu
def test_gpu_c5_full_size(built):
    """C5 at its configs[4] size: 256K 8x8 tiles of a 4096^2 image, 50 iterations. This
    batch (4096 waves) selects the LDS-frame threaded core. Every 7th tile against the
    oracle exactly (f64 results, 64-bit masks, rendered bytes in the memory hash)."""
    wasm = W.mandel_wasm()
    n = 262144
    rows = [[i, 4096, 50] for i in range(n)]
    rets, st, cnt, h = gpu_run(wasm, "tile", rows, [I32, I32, I32], [I64])
    assert all(int(s) == 0 for s in st)
    idx = list(range(0, n, 7))
    ref = _oracle_batch(wasm, "tile", [rows[i] for i in idx])
    sub = lambda a: [a[i] for i in idx]
    assert compare(ref, sub(rets), sub(st), sub(cnt), sub(h), [I64], exact=True) == []


@pytest.mark.gpu
@pytest.mark.parametrize("granule", [4, 8, 16, 128])
def test_gpu_memory_granules_bit_exact(built, granule):
    """The memory interleave granule is layout only (MemoryGranule, dbc_ops.h GMem): every
    workload -- uniform (BLAKE3, Mandelbrot) and per-lane (quicksort, Collatz) addresses,
    i64 / v128 / byte accesses, memory.grow zeroing -- and the memory hash are identical
    at every granule."""
    cases = _cases()
    wasm, func, pt, rt, _ = cases["qsort"]
    cases["qsort"] = (wasm, func, pt, rt, [[i, (i * 37) % 700] for i in range(130)])
    for name in ("blake3", "qsort", "collatz", "mandel"):
        wasm, func, pt, rt, rows = cases[name]
        ref = oracle_run(O.Module(wasm), func, rows)
        got = gpu_run(wasm, func, rows, pt, rt, memory_granule=granule)
        assert compare(ref, *got, rt, exact=True) == [], name


# Partial waves: a batch whose last wave is not full (8 lanes: one
# partial wave; 65: a full wave and a 1-lane wave) through every engine. The lanes past
# NumInstances are never running (batch_kernel.hip: status OK from the start), so no engine
# may read their params, frames or memory or write their results. (Round 2's only GPU fault,
# gpurun_out/g3, hit an 8-lane batch while the SIMT core was being built: see DESIGN.md
# "Partial waves".)
ENGINES = {
    "simt": {},                                   # V frames, compiled runs, SIMT scheduling
    "trip": {"WB_TRIP": "1"},                     # V frames, trip mode
    "nosimt": {"WB_SIMT": "0"},                   # V frames, compiled runs without SIMT
    "nojit": {"WB_JIT": "0"},                     # V frames, threaded core handlers only
    "lds": {"WB_VFRAME": "0"},                    # LDS frames, threaded core
    "step": {"WB_THREADED": "0"},                 # the compiled C++ step only
    "hbm": {"WB_HBMFRAME": "1"},                  # frames in HBM (compiled step)
}


@pytest.mark.gpu
@pytest.mark.parametrize("engine", sorted(ENGINES))
@pytest.mark.parametrize("n", [8, 65])
def test_gpu_partial_waves_every_engine(built, monkeypatch, engine, n):
    for k, v in ENGINES[engine].items():
        monkeypatch.setenv(k, v)
    fib = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fibonacci.wasm"), "rb").read()
    cases = {
        "fib": (fib, "fib", [I32], [I32], [[(i * 7) % 19] for i in range(n)]),
        "qsort": (W.qsort_wasm(), "sort", [I32, I32], [I32], [[i, (i * 37) % 300] for i in range(n)]),
        "collatz": (W.collatz_wasm(), "collatz", [I32, I32], [I32],
                    [[i * 89 if i % 5 == 0 else i, 10000] for i in range(n)]),
        "mandel": (W.mandel_wasm(), "tile", [I32, I32, I32], [I64], [[i * 5, 128, 50] for i in range(n)]),
    }
    for name, (wasm, func, pt, rt, rows) in cases.items():
        ref = oracle_run(O.Module(wasm), func, rows)
        rets, st, cnt, h = gpu_run(wasm, func, rows, pt, rt)
        assert compare(ref, rets, st, cnt, h, rt) == [], (engine, name)
