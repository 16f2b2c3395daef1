"""Host-function cost under gas metering.

The reference charges a host function's cost when it is called, after its frame is pushed
and before it runs: `Stat->addCost(HostFunc.getCost())` fails with CostLimitExceeded
(0x03) when the total would pass the limit (lib/executor/helper.cpp:59-64); the cost is
the one given to WasmEdge_FunctionInstanceCreate(Type, Func, Data, Cost)
(include/api/wasmedge/wasmedge.h:2324, include/runtime/hostfunc.h:28-46). The call
instruction itself is counted and priced first by the dispatch loop (engine.cpp:1616-1630).

The batched path takes the cost in WasmEdge_BatchAddHostFunctionWithCost and charges it in
the host service round, before the host function runs (hostcall.cpp); the oracle restates
the rule (oracle/wasm_oracle_exec.inc enter_function_t). Checked: status, instruction
count, memory hash and the gas total, for limits that trip on ordinary instructions and
exactly at a host call, with direct calls, call_indirect and a return_call from the entry
function (the tail-call shape on which the batched path and the reference agree,
tests/test_tailcall.py)."""
import pytest

import oracle_py as O
from helpers import compare
from wasmedge_amd.wat import assemble

I32, I64 = 0x7F, 0x7E
COSTS = {("env", "add_i64"): 5, ("env", "mem_sum"): 7}

HOSTCOST = assemble(r"""
(module
  (import "env" "add_i64" (func $add (param i64 i64) (result i64)))
  (import "env" "mem_sum" (func $sum (param i32 i32) (result i32)))
  (type $tsum (func (param i32 i32) (result i32)))
  (table 1 funcref)
  (elem (i32.const 0) $sum)
  (memory 1)
  (func (export "run") (param $iid i32) (result i64)
    (local $i i32) (local $acc i64)
    (i32.store (i32.const 0) (local.get $iid))
    (loop $l
      (local.set $acc (call $add (local.get $acc) (i64.extend_i32_u (local.get $i))))
      (local.set $acc (i64.add (local.get $acc)
        (i64.extend_i32_u (call $sum (i32.const 0) (i32.const 4)))))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $i)
        (i32.add (i32.rem_u (local.get $iid) (i32.const 4)) (i32.const 1)))))
    (local.set $acc (i64.add (local.get $acc) (i64.extend_i32_u
      (call_indirect (type $tsum) (i32.const 0) (i32.const 2) (i32.const 0)))))
    (i32.store (i32.const 8) (i32.wrap_i64 (local.get $acc)))
    (return_call $add (local.get $acc) (i64.const 3))))
""")

ROWS = [[i] for i in range(64)]


def _oracle(limit, costs=COSTS, rows=ROWS):
    """[(code, results, count, hash)], [gas total] of a fresh metered instance per row;
    (None, None) when the instantiation itself runs out of gas."""
    O.set_host_costs(costs)
    try:
        m = O.Module(HOSTCOST, tail_call=True)
        insts = [O.Instance(m, cost_limit=limit) for _ in rows]
        if not insts[0]._h:
            assert insts[0].error == 0x03
            return None, None
        ref = [x.invoke("run", r) for x, r in zip(insts, rows)]
        return ref, [x.cost_sum() for x in insts]
    finally:
        O.set_host_costs({})


BIG = 1 << 62


def _host_trip_limits(row):
    """Limits at which `row` stops exactly at a host call: the count stays put while the
    limit rises through the host function's cost (the call instruction was counted and
    priced, the host cost did not fit)."""
    _, full = _oracle(BIG, rows=[row])
    out = []
    prev = None
    for limit in range(1, full[0] + 1):
        ref, _ = _oracle(limit, rows=[row])
        if ref is None:
            continue
        code, _, cnt, _ = ref[0]
        if code == 0x03 and prev is not None and prev[0] == 0x03 and prev[2] == cnt:
            out.append(limit)
        prev = ref[0]
    return out, full[0]


def test_oracle_host_cost_rule():
    """The oracle's restatement: the gas total of a run is its instructions' unit costs
    plus 5 per add_i64 call and 7 per mem_sum call; a limit inside a host function's cost
    stops the instance at that call (count unchanged across the window, status 0x03)."""
    ref0, cost0 = _oracle(BIG, costs={})
    ref1, cost1 = _oracle(BIG)
    for (c0, v0, n0, h0), (c1, v1, n1, h1), a, b, r in zip(ref0, ref1, cost0, cost1, ROWS):
        assert c0 == c1 == 0 and v0 == v1 and n0 == n1 and h0 == h1
        calls = r[0] % 4 + 1
        # loop: add + sum per trip; call_indirect -> sum; the tail call -> add
        assert b - a == calls * (5 + 7) + 7 + 5, r
        assert a >= n0   # unit costs: one per counted instruction (+ instantiation)
    trips, full = _host_trip_limits([2])
    # add_i64 (5) and mem_sum (7) windows: 4 and 6 limits each where the count stays put
    assert len(trips) >= 4 + 6, trips


@pytest.mark.gpu
def test_gpu_host_cost_metering(built):
    """64 lanes (1..4 loop trips each), limits over the whole range -- including every
    limit inside the host-cost windows of the first calls -- bit-exact against the
    oracle: status, count, memory hash, gas total."""
    from hostfuncs import ENV
    from wasmedge_amd import batch
    _, full = _oracle(BIG)
    trips, _ = _host_trip_limits([3])
    limits = sorted(set([1, 2, 17, max(full) // 3, max(full) // 2, min(full) - 1, min(full),
                         max(full) - 1, max(full), max(full) + 1, BIG] + trips[:24]))
    for limit in limits:
        ref, rcost = _oracle(limit)
        if ref is None:   # the instantiation (the elem offset) runs out of gas
            with pytest.raises(batch.WasmEdgeError) as e:
                batch.BatchContext(HOSTCOST, len(ROWS), device=0, cost_limit=limit, tail_call=True)
            assert e.value.code == 0x03
            continue
        ctx = batch.BatchContext(HOSTCOST, len(ROWS), device=0, cost_limit=limit, tail_call=True)
        try:
            for (mod, name), c in COSTS.items():
                fn, np_, nr = ENV[name]
                ctx.add_host_function(mod, name, fn, np_, nr, cost=c)
            rets, st, cnt = ctx.execute("run", batch.make_values(ROWS, [I32]), 1)
            ints = batch.ret_ints(rets)
            got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(ROWS))]
            assert compare(ref, got, st, cnt, ctx.memory_hash(), [I64]) == [], limit
            assert [int(c) for c in ctx.total_costs()] == rcost, limit
        finally:
            ctx.close()


@pytest.mark.gpu
def test_gpu_host_cost_ignored_without_metering(built):
    """Without a CostLimit the batch does not meter: host costs change nothing and the
    gas totals read 0 (WasmEdge_BatchGetTotalCosts)."""
    from hostfuncs import ENV
    from wasmedge_amd import batch
    ref, _ = _oracle(0)
    ctx = batch.BatchContext(HOSTCOST, len(ROWS), device=0, tail_call=True)
    try:
        for (mod, name), c in COSTS.items():
            fn, np_, nr = ENV[name]
            ctx.add_host_function(mod, name, fn, np_, nr, cost=c)
        rets, st, cnt = ctx.execute("run", batch.make_values(ROWS, [I32]), 1)
        ints = batch.ret_ints(rets)
        got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(ROWS))]
        assert compare(ref, got, st, cnt, ctx.memory_hash(), [I64]) == []
        assert not ctx.total_costs().any()
    finally:
        ctx.close()
