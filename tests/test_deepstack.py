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
    waves: bit-exact against the oracle (returns, counts, memory), twice (each Reset gives
    the growth back and the second run grows the stack again)."""
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


# a runaway recursion, then a memory.grow-heavy run and a deep finite recursion on the same
# context (the stack's growth is bounded by CallStackMaxBytes and given back at
# Reset, and Reset re-arms it, so memory growth after it still finds the device memory and
# the next deep recursion grows the stack again)
RUNAWAY = assemble(r"""
(module
  (memory 1)
  (func $down (param $n i32) (result i32)
    (i32.add (i32.const 1) (call $down (i32.add (local.get $n) (i32.const 1)))))
  (func $sum (param $n i32) (result i32)
    (if (result i32) (i32.eqz (local.get $n))
      (then (i32.const 0))
      (else (i32.add (local.get $n) (call $sum (i32.sub (local.get $n) (i32.const 1)))))))
  (func (export "runaway") (param $n i32) (result i32) (call $down (local.get $n)))
  (func (export "sum") (param $n i32) (result i32) (call $sum (local.get $n)))
  (func (export "grow") (param $n i32) (result i32)
    (local $p i32)
    (local.set $p (memory.grow (local.get $n)))
    (if (i32.ge_s (local.get $p) (i32.const 0))
      (then (i32.store (i32.sub (i32.shl (memory.size) (i32.const 16)) (i32.const 4))
                       (i32.add (local.get $n) (i32.const 7)))))
    (i32.add (i32.mul (local.get $p) (i32.const 1000)) (memory.size))))
""")


@pytest.mark.gpu
def test_gpu_runaway_recursion_then_reset_then_grow(built):
    from wasmedge_amd import batch
    n = 64

    def check(ctx, func, rows):
        ref = []
        for r in rows:                       # (a fresh instance per row, as after a Reset)
            ref.append(O.Module(RUNAWAY).run(func, r))
        rets, st, cnt = ctx.execute(func, batch.make_values(rows, [I32]), 1)
        ints = batch.ret_ints(rets)
        got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(n)]
        assert compare(ref, got, st, cnt, ctx.memory_hash(), [I32]) == [], func

    ctx = batch.BatchContext(RUNAWAY, n, device=0, call_stack_max_bytes=64 << 20)
    try:
        _, st, cnt = ctx.execute("runaway", batch.make_values([[i] for i in range(n)], [I32]), 1)
        assert set(int(x) for x in st) == {0xB0}         # the bound, not the whole device
        ctx.reset()
        check(ctx, "grow", [[300 + 11 * i] for i in range(n)])
        ctx.reset()
        check(ctx, "sum", [[20000 + i] for i in range(n)])   # ~40K cells: grows again
        ctx.reset()
        check(ctx, "sum", [[20000 + 3 * i] for i in range(n)])
    finally:
        ctx.close()
