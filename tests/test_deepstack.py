"""The call stack grows on demand. The reference's value and frame
stacks are std::vectors that grow without bound (include/runtime/stackmgr.h:44-47). The
batched path reserves 4096 cells per instance and, when a call would pass them
(CallStackCells 0, the default), parks the lane at the call, doubles the stack between
launches (hostcall.cpp grow_stack) and runs the call again -- counted once, so counts stay
exact. A fixed CallStackCells keeps the old bound (0xB0 past it; tests/test_scalar.py)."""
import pytest

import oracle_py as O
from helpers import compare
from wasmedge_amd.wat import assemble

I32 = 0x7F

# sum(n) = n + sum(n - 1) by plain recursion (no tail call): every frame spills its
# parameter and a return record, so depth n takes ~2n call-stack cells
DEEP = assemble(r"""
(module
  (memory 1)
  (func $sum (param $n i32) (result i32)
    (if (result i32) (i32.eqz (local.get $n))
      (then (i32.const 0))
      (else (i32.add (local.get $n) (call $sum (i32.sub (local.get $n) (i32.const 1)))))))
  (func (export "run") (param $n i32) (result i32)
    (i32.store (i32.const 16) (call $sum (local.get $n)))
    (i32.load (i32.const 16))))
""")


def test_oracle_deep_recursion():
    m = O.Module(DEEP)
    code, vals, cnt, _ = m.run("run", [50000])
    assert code == 0 and vals == [(50000 * 50001 // 2) & 0xFFFFFFFF]


@pytest.mark.gpu
@pytest.mark.parametrize("n_lanes", [64, 192])
def test_gpu_recursion_20x_the_default_stack(built, n_lanes):
    """Recursion 41,000+ frames deep (over 80,000 cells: more than 20x the 4096-cell
    default reservation) on every lane, depths differing per lane, over one and three
    waves: bit-exact against the oracle (returns, counts, memory), twice (the grown stack
    stays)."""
    from wasmedge_amd import batch
    rows = [[41000 + 37 * i] for i in range(n_lanes)]
    m = O.Module(DEEP)
    ref = [m.run("run", r) for r in rows]
    ctx = batch.BatchContext(DEEP, n_lanes, device=0)
    try:
        for rep in range(2):
            rets, st, cnt = ctx.execute("run", batch.make_values(rows, [I32]), 1)
            ints = batch.ret_ints(rets)
            got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(n_lanes)]
            assert compare(ref, got, st, cnt, ctx.memory_hash(), [I32]) == [], rep
            ctx.reset()
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_fixed_stack_still_bounded(built):
    """An explicit CallStackCells stays a fixed bound: past it the lane ends with 0xB0."""
    from wasmedge_amd import batch
    ctx = batch.BatchContext(DEEP, 64, device=0, call_stack_cells=4096)
    try:
        rets, st, cnt = ctx.execute("run", batch.make_values([[41000]] * 64, [I32]), 1)
        assert all(int(s) == 0xB0 for s in st)
    finally:
        ctx.close()
