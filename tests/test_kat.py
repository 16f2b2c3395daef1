"""Known-answer tests pinned by the reference's own fixtures.

* tools/wasmedge/examples/README.md: fib 8 -> 34, fac 12 -> 479001600
* test/thread/ThreadTest.cpp:152-169: four mt19937 answers (i64 + SIMD128 + memory)
* fib(30) = 1346269 with 28,271,634 counted instructions (measured on the reference,
  SURVEY.md section 0 / BASELINE.md section 2)
"""
import json

import pytest

import oracle_py as O
from conftest import golden
from helpers import compare, emu_run, gpu_run, oracle_run

I32, I64 = 0x7F, 0x7E


def _mt_rows():
    j = json.loads(golden("mt19937.json", "r"))
    return j["args"], j["answers"]


def test_oracle_kats(built):
    fib = O.Module(golden("fibonacci.wasm"))
    assert fib.run("fib", [8])[1] == [34]
    code, vals, cnt, _ = fib.run("fib", [30])
    assert (code, vals, cnt) == (0, [1346269], 28271634)
    assert O.Module(golden("factorial.wasm")).run("fac", [12])[1] == [479001600]
    mt = O.Module(golden("mt19937.wasm"))
    args, answers = _mt_rows()
    for a, ans in zip(args, answers):
        code, vals, cnt, _ = mt.run("mt19937", a)
        assert code == 0 and vals == [ans]
        assert cnt == 2095253      # reference count (SURVEY.md 8c "Verified outputs")


def test_emulator_kats(built):
    """The kernel's own step code (dbc_step.inc) run on the host over the lowering."""
    fib = golden("fibonacci.wasm")
    rets, st, cnt, _ = emu_run(fib, "fib", [[8], [30]], [I32], [I32])
    assert rets == [[34], [1346269]] and list(cnt) == [699, 28271634]
    args, answers = _mt_rows()
    rets, st, cnt, _ = emu_run(golden("mt19937.wasm"), "mt19937", args, [I32, I64, I64], [I64])
    assert [r[0] for r in rets] == answers and set(cnt.tolist()) == {2095253}


@pytest.mark.gpu
def test_gpu_fib_kat(built):
    rows = [[8], [30], [0], [1], [2]]
    rets, st, cnt, h = gpu_run(golden("fibonacci.wasm"), "fib", rows, [I32], [I32])
    assert rets == [[34], [1346269], [1], [1], [2]]
    assert int(cnt[1]) == 28271634


@pytest.mark.gpu
def test_gpu_fac_kat(built):
    rets, st, cnt, h = gpu_run(golden("factorial.wasm"), "fac", [[12], [5]], [I32], [I32])
    assert rets == [[479001600], [120]]


@pytest.mark.gpu
def test_gpu_mt19937_kat(built):
    args, answers = _mt_rows()
    wasm = golden("mt19937.wasm")
    rets, st, cnt, h = gpu_run(wasm, "mt19937", args, [I32, I64, I64], [I64])
    assert [r[0] for r in rets] == answers
    assert set(int(c) for c in cnt) == {2095253}
    ref = oracle_run(O.Module(wasm), "mt19937", args)
    assert compare(ref, rets, st, cnt, h, [I64]) == []


@pytest.mark.gpu
def test_gpu_fib_64k_divergent(built):
    """SURVEY 8d C1 plumbing variant: 64K lanes, n_i = 20 + (i mod 11) -> recursion depth
    and trip counts diverge inside every wavefront."""
    n = 65536
    rows = [[20 + (i % 11)] for i in range(n)]
    rets, st, cnt, h = gpu_run(golden("fibonacci.wasm"), "fib", rows, [I32], [I32])
    fibm = O.Module(golden("fibonacci.wasm"))
    ref = {k: fibm.run("fib", [k]) for k in range(20, 31)}
    assert all(int(s) == 0 for s in st)
    for i in range(n):
        k = 20 + (i % 11)
        assert rets[i] == ref[k][1] and int(cnt[i]) == ref[k][2], i



@pytest.mark.gpu
@pytest.mark.parametrize("jit", ["1", "0"])
def test_gpu_mt19937_per_instance_seeds(built, monkeypatch, jit):
    """bench.py's `mt` workload (a second real module through the
    compiled runs, whose v128 loads/stores, bitselect and i64x2 shifts now compile): 4,096
    instances each drawing 3,000 numbers from its own seed, against the oracle on a sample,
    with the compiled runs on and off."""
    monkeypatch.setenv("WB_JIT", jit)
    wasm = golden("mt19937.wasm")
    n = 4096
    rows = [[0, 5489 + i, 3000] for i in range(n)]
    rets, st, cnt, h = gpu_run(wasm, "mt19937", rows, [I32, I64, I64], [I64])
    idx = list(range(0, n, 37)) + [n - 1]
    ref = oracle_run(O.Module(wasm), "mt19937", [rows[i] for i in idx])
    assert compare(ref, [rets[i] for i in idx], [st[i] for i in idx], [cnt[i] for i in idx],
                   [h[i] for i in idx], [I64]) == []
