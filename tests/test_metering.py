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
    """The default unit table (every instruction costs 1)."""
    _gpu_sweep(name, None)


@pytest.mark.gpu
@pytest.mark.parametrize("trip", ["0", "1"])
def test_gpu_interrupt(built, monkeypatch, trip):
    """An endless loop on 64K lanes stops with Interrupted (0x07) when another thread
    calls WasmEdge_BatchInterrupt, within 100 ms of the call (the kernel polls the flag
    every scheduler round and a core call returns at least every 2^20 instructions; the
    reference checks its StopToken on every branch: helper.cpp:184-187), with SIMT
    scheduling and in trip mode."""
    monkeypatch.setenv("WB_TRIP", trip)
    from wasmedge_amd import batch
    from wasmedge_amd.wat import assemble
    spin = assemble("(module (func (export \"spin\") (param i32) (result i32)"
                    " (loop $l (local.set 0 (i32.add (local.get 0) (i32.const 1))) (br $l))"
                    " (local.get 0))"
                    " (func (export \"count\") (param i32) (result i32) (local i32)"
                    " (loop $l (local.set 1 (i32.add (local.get 1) (i32.const 1)))"
                    " (br_if $l (i32.lt_u (local.get 1) (local.get 0)))) (local.get 1)))")
    ctx = batch.BatchContext(spin, 65536, device=0, time_limit=60.0)
    try:
        asked = []

        def stop():
            asked.append(time.perf_counter())
            ctx.interrupt()
        t = threading.Timer(1.0, stop)
        t.start()
        rets, st, cnt = ctx.execute("spin", batch.make_values([[i] for i in range(65536)], [I32]), 1)
        latency = time.perf_counter() - asked[0]
        t.join()
        assert all(int(s) == 0x07 for s in st)
        assert latency < 0.1, latency
        # the interrupt ends that run only: the next one runs to completion
        ctx.reset()
        rets, st, cnt = ctx.execute("count", batch.make_values([[2000]] * 65536, [I32]), 1)
        assert all(int(s) == 0 for s in st) and len(set(int(c) for c in cnt)) == 1
        assert int(cnt[0]) > 2000
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("trip", ["0", "1"])
def test_gpu_max_steps_is_tight(built, monkeypatch, trip):
    """MaxSteps: a lane stops (Interrupted) once its count reaches the budget, past it by
    less than one compiled run (the core's budget per call is the smallest remaining budget
    of the running lanes), whatever each lane had retired before."""
    monkeypatch.setenv("WB_TRIP", trip)
    from wasmedge_amd import batch
    from wasmedge_amd.wat import assemble
    spin = assemble("(module (func (export \"spin\") (param i32) (result i32)"
                    " (loop $l (br_if $l (i32.and (i32.const 1) (i32.gt_u (local.get 0) (i32.const 7))))"
                    "   (local.set 0 (i32.add (local.get 0) (i32.const 1))) (br $l))"
                    " (local.get 0)))")
    for budget in (1000, 123457):
        ctx = batch.BatchContext(spin, 4096, device=0, max_steps=budget)
        try:
            rets, st, cnt = ctx.execute("spin", batch.make_values([[i % 13] for i in range(4096)], [I32]), 1)
            assert all(int(s) == 0x07 for s in st)
            over = [int(c) - budget for c in cnt]
            assert min(over) >= 0 and max(over) < 16, (budget, min(over), max(over))
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


# ---- custom cost tables (WasmEdge_StatisticsSetCostTable, statistics.h:32,59-66,
# lib/api/wasmedge.cpp:878-882): every instruction adds CostTab[OpCode]; the first one that
# would take the instance's running total past the limit fails with CostLimitExceeded,
# counted and unpriced. The total runs on from instantiation across invocations.
import random  # noqa: E402

BIG = 1 << 62


def _tables():
    """The reference API test's table (test/api/APIUnitTest.cpp:1067-1072: 512 x 20, the
    rest 0 -- every SIMD and most prefixed ops are free), and random tables with zeros."""
    rng = random.Random(7)
    out = {"apitest": [20] * 512}
    for k in range(2):
        t = [0] * 65536
        for op in list(range(0x100)) + list(range(0xFC00, 0xFC12)) + list(range(0xFD00, 0xFE00)):
            t[op] = rng.choice([0, 0, 1, 2, 3, 5, 17, 100])
        out["random%d" % k] = t
    return out


TABLES = _tables()


def _oracle_tab(wasm, func, rows, limit, table):
    m = O.Module(wasm)
    out, costs = [], []
    for r in rows:
        inst = O.Instance(m, cost_limit=limit, cost_table=table)
        out.append(inst.invoke(func, r))
        costs.append(inst.cost_sum() if not inst.error else None)   # None: instantiation failed
    return out, costs


@pytest.mark.parametrize("tab", sorted(TABLES))
@pytest.mark.parametrize("name", sorted(CASES))
def test_cost_table_sweep_emulator(built, name, tab):
    wasm, func, pt, rt, rows = CASES[name]
    table = TABLES[tab]
    _, full = _oracle_tab(wasm, func, rows, BIG, table)
    total = max(full)
    step = max(1, total // 150)
    for limit in sorted(set(list(range(1, total + 2, step)) + [total - 1, total, total + 1])):
        if limit <= 0:
            continue
        ref, rcost = _oracle_tab(wasm, func, rows, limit, table)
        costs = []
        rets, st, cnt, h = emu_run(wasm, func, rows, pt, rt, cost_limit=limit, cost_table=table,
                                   costs_out=costs)
        bad = compare(ref, rets, st, cnt, h, rt)
        assert bad == [], (limit, bad[:3])
        assert [c for c, r in zip(costs, rcost) if r is not None] == \
            [r for r in rcost if r is not None], limit


def test_cost_accumulates_across_invocations(built):
    """The gas total is the instance's, not the invocation's: a second run on the same
    instance starts from where the first stopped (Statistics::CostSum is cleared only by
    VM cleanup, lib/vm/vm.cpp:336-340)."""
    m = O.Module(STATEFUL)
    inst = O.Instance(m, cost_limit=BIG, cost_table=TABLES["random0"])
    start = inst.cost_sum()
    assert start > 0                                   # constant exprs + start function
    a = inst.invoke("step", [4]); c1 = inst.cost_sum()
    b = inst.invoke("step", [4]); c2 = inst.cost_sum()
    assert a[0] == b[0] == 0 and c1 > start and c2 > c1


@pytest.mark.gpu
@pytest.mark.parametrize("tab", sorted(TABLES))
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_cost_table(built, name, tab):
    """Device vs oracle under a custom cost table at limits across the program: status,
    count, memory hash and each instance's gas total."""
    _gpu_sweep(name, TABLES[tab])


def _gpu_sweep(name, table):
    from wasmedge_amd import batch
    wasm, func, pt, rt, rows = CASES[name]
    _, full = _oracle_tab(wasm, func, rows, BIG, table)
    total = max(full)
    for limit in sorted({1, 2, total // 3, total // 2, total - 1, total, total + 5, BIG}):
        if limit <= 0:
            continue
        ref, rcost = _oracle_tab(wasm, func, rows, limit, table)
        if any(c is None for c in rcost):     # instantiation itself runs out of gas
            with pytest.raises(batch.WasmEdgeError) as e:
                batch.BatchContext(wasm, len(rows), device=0, cost_limit=limit, cost_table=table)
            assert e.value.code == 0x03
            continue
        ctx = batch.BatchContext(wasm, len(rows), device=0, cost_limit=limit, cost_table=table)
        try:
            rets, st, cnt = ctx.execute(func, batch.make_values(rows, pt), len(rt))
            ints = batch.ret_ints(rets)
            got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(rows))]
            assert compare(ref, got, st, cnt, ctx.memory_hash(), rt) == [], limit
            assert [int(c) for c in ctx.total_costs()] == rcost, limit
        finally:
            ctx.close()


@pytest.mark.gpu
def test_gpu_cost_runs_on_across_invocations(built):
    from wasmedge_amd import batch
    table = TABLES["random1"]
    rows = [[4], [1], [3]]
    m = O.Module(STATEFUL)
    insts = [O.Instance(m, cost_limit=BIG, cost_table=table) for _ in rows]
    ctx = batch.BatchContext(STATEFUL, len(rows), device=0, cost_limit=BIG, cost_table=table)
    try:
        assert [int(c) for c in ctx.total_costs()] == [i.cost_sum() for i in insts]
        for _ in range(3):
            ctx.execute("step", batch.make_values(rows, [I32]), 1)
            for i, r in zip(insts, rows):
                i.invoke("step", r)
            assert [int(c) for c in ctx.total_costs()] == [i.cost_sum() for i in insts]
    finally:
        ctx.close()


METER_JIT = {
    "blake3": (W.blake3_wasm(), "run", [I32, I32], [I32], [[5, 2], [9, 1]]),
    "fib": CASES["fib"][:4] + ([[7], [9]],),
    "qsort": CASES["qsort"],
}


@pytest.mark.gpu
@pytest.mark.parametrize("tab", [None, "random0"])
@pytest.mark.parametrize("name", sorted(METER_JIT))
def test_gpu_metered_compiled_runs(built, name, tab):
    """Metered contexts run the module's compiled runs (jit.cpp prices each run at entry
    against the limit and adds the exact price of the way it leaves): a dense limit sweep
    so the limit falls inside, at the start and at the end of runs, calls and returns."""
    from wasmedge_amd import batch
    wasm, func, pt, rt, rows = METER_JIT[name]
    table = TABLES[tab] if tab else None
    _, full = _oracle_tab(wasm, func, rows, BIG, table)
    total = max(full)
    runs = 0
    limits = sorted(set(list(range(1, total + 2, max(1, total // 60))) + [total - 1, total, total + 1]))
    for limit in limits:
        if limit <= 0:
            continue
        ref, rcost = _oracle_tab(wasm, func, rows, limit, table)
        if any(c is None for c in rcost):
            continue
        ctx = batch.BatchContext(wasm, len(rows), device=0, cost_limit=limit, cost_table=table)
        try:
            runs = max(runs, ctx.compiled_runs())
            rets, st, cnt = ctx.execute(func, batch.make_values(rows, pt), len(rt))
            ints = batch.ret_ints(rets)
            got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(rows))]
            assert compare(ref, got, st, cnt, ctx.memory_hash(), rt) == [], limit
            assert [int(c) for c in ctx.total_costs()] == rcost, limit
        finally:
            ctx.close()
    assert runs > 0
