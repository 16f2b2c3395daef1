"""Gas metering: the reference's unit-cost limit (statistics.h:69-91,
engine.cpp:1616-1630, controlInstr.cpp:23-28) is exact -- an instance executes CostLimit
instructions and the next one fails with CostLimitExceeded (0x03), counted. The limit is
swept over every value up to a program's full count, so the trap lands on every kind of
instruction (folded, fused, branch landings, else, calls, returns), and checked against
the oracle: status, count, and the memory hash (no partial side effects past the limit).
Also: the host-settable interrupt (WasmEdge_BatchInterrupt)."""
import threading
import time

import pytest

import oracle_py as O
from conftest import golden
from helpers import compare, emu_run
from test_instance import STATEFUL
from wasmedge_amd import workloads as W

I32, I64 = 0x7F, 0x7E


def _oracle(wasm, func, rows, limit):
    m = O.Module(wasm)
    return [O.Instance(m, cost_limit=limit).invoke(func, r) for r in rows]


CASES = {
    "fib": (golden("fibonacci.wasm"), "fib", [I32], [I32], [[6]]),
    "collatz": (W.collatz_wasm(), "collatz", [I32, I32], [I32], [[7, 10000]]),
    "qsort": (W.qsort_wasm(), "sort", [I32, I32], [I32], [[3, 12]]),
    "stateful": (STATEFUL, "step", [I32], [I32], [[4], [1], [3]]),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_cost_limit_sweep_emulator(built, name):
    wasm, func, pt, rt, rows = CASES[name]
    full = max(r[2] for r in _oracle(wasm, func, rows, 0))
    step = max(1, full // 400)
    for limit in list(range(1, full + 2, step)) + [full - 1, full, full + 1]:
        if limit <= 0:
            continue
        ref = _oracle(wasm, func, rows, limit)
        rets, st, cnt, h = emu_run(wasm, func, rows, pt, rt, cost_limit=limit)
        bad = compare(ref, rets, st, cnt, h, rt)
        assert bad == [], (limit, bad[:3])
        if limit <= full - 1:
            assert all(r[0] == 0x03 and r[2] == limit + 1 for r in ref if r[2] > limit)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_cost_limit(built, name):
    from helpers import gpu_run
    wasm, func, pt, rt, rows = CASES[name]
    full = max(r[2] for r in _oracle(wasm, func, rows, 0))
    for limit in sorted({1, 2, 3, full // 3, full // 2, full - 1, full, full + 5}):
        if limit <= 0:
            continue
        ref = _oracle(wasm, func, rows, limit)
        got = gpu_run(wasm, func, rows, pt, rt, cost_limit=limit)
        assert compare(ref, *got, rt) == [], limit


@pytest.mark.gpu
def test_gpu_interrupt(built):
    """An endless loop on 64K lanes stops with Interrupted (0x07) when another thread
    calls WasmEdge_BatchInterrupt."""
    from wasmedge_amd import batch
    from wasmedge_amd.wat import assemble
    spin = assemble("(module (func (export \"spin\") (param i32) (result i32)"
                    " (loop $l (local.set 0 (i32.add (local.get 0) (i32.const 1))) (br $l))"
                    " (local.get 0)))")
    ctx = batch.BatchContext(spin, 65536, device=0, time_limit=60.0)
    try:
        t = threading.Timer(1.0, ctx.interrupt)
        t.start()
        t0 = time.time()
        rets, st, cnt = ctx.execute("spin", batch.make_values([[i] for i in range(65536)], [I32]), 1)
        t.join()
        assert time.time() - t0 < 30
        assert all(int(s) == 0x07 for s in st)
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_interrupt_reference_module(built):
    """The reference's interrupt test module (test/executor/ExecutorTest.cpp:118-146,
    fixture tests/golden/executor_interrupt.wasm: `_start` = loop br 0): still running
    after 1 ms, then cancelled -> every lane Interrupted (0x07)."""
    from wasmedge_amd import batch
    from conftest import golden
    ctx = batch.BatchContext(golden("executor_interrupt.wasm"), 4096, device=0, time_limit=60.0)
    try:
        t = threading.Timer(0.5, ctx.interrupt)
        t.start()
        t0 = time.time()
        rets, st, cnt = ctx.execute("_start", batch.make_values([[]] * 4096, []), 0)
        t.join()
        assert time.time() - t0 >= 0.001 and time.time() - t0 < 30
        assert all(int(s) == 0x07 for s in st)
        assert all(int(c) > 1000 for c in cnt)
    finally:
        ctx.close()
