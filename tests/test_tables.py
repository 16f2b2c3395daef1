"""Tables: per-lane mutable tables -- table.get/set/size/grow/fill/
copy/init, elem.drop, several tables, an externref table, passive/declarative element
segments and call_indirect through a table the lane has changed. Expected values: the
oracle (oracle_py), which follows lib/executor/engine/tableInstr.cpp,
include/runtime/instance/table.h (getRefAddr :131, growTable, setInitList) and
controlInstr.cpp:101-158; its table semantics are pinned by the reference's own
test/spec fixtures only through the spec suite, so the cases here are parity against the
restatement (parity unpinned beyond it)."""
import pytest

import oracle_py as O
from helpers import compare, emu_run
from wasmedge_amd.wat import assemble

I32 = 0x7F

TABLES = assemble(r"""
(module
  (type $ii (func (param i32) (result i32)))
  (table $t 4 16 funcref)
  (table $u 2 externref)
  (table $w 3 funcref)
  (func $f0 (type $ii) (i32.add (local.get 0) (i32.const 1)))
  (func $f1 (type $ii) (i32.mul (local.get 0) (i32.const 3)))
  (func $f2 (type $ii) (i32.sub (local.get 0) (i32.const 7)))
  (func $f3 (param i64) (result i64) (local.get 0))
  (elem (table $t) (i32.const 0) func $f0 $f1)
  (elem $p func $f2 $f1 $f0 $f3)
  (elem $q funcref (ref.func $f2) (ref.null func))
  (elem declare func $f3)
  (elem (table $w) (i32.const 1) func $f2 $f0)
  (func (export "run") (param $x i32) (result i32)
    (local $r i32)
    (if (i32.and (local.get $x) (i32.const 1))
      (then (table.set $t (i32.const 2) (ref.func $f2))))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 3)) (i32.const 0))
      (then (local.set $r (table.grow $t (ref.func $f1) (i32.rem_u (local.get $x) (i32.const 5))))))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 7)) (i32.const 2))
      (then (elem.drop $p)))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 4)) (i32.const 1))
      (then (table.init $t $p (i32.const 1) (i32.and (i32.shr_u (local.get $x) (i32.const 2)) (i32.const 1)) (i32.const 3))))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 6)) (i32.const 5))
      (then (table.copy $t $t (i32.const 0) (i32.const 1) (i32.const 3))))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 9)) (i32.const 4))
      (then (table.copy $t $t (i32.const 1) (i32.const 0) (i32.const 3))))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 8)) (i32.const 7))
      (then (table.fill $t (i32.const 1) (ref.null func) (i32.const 2))))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 10)) (i32.const 3))
      (then (table.init $w $q (i32.const 0) (i32.const 0) (i32.const 2))))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 11)) (i32.const 6))
      (then (table.copy $w $t (i32.const 0) (i32.const 0) (i32.const 3))))
    (if (i32.eq (local.get $x) (i32.const 20))
      (then (table.fill $t (i32.const 3) (ref.func $f0) (i32.const 9))))
    (if (i32.eq (local.get $x) (i32.const 22))
      (then (drop (table.get $u (i32.const 2)))))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 5)) (i32.const 2))
      (then (table.set $u (i32.const 1) (table.get $u (i32.const 0)))))
    (local.set $r (i32.add (local.get $r)
      (i32.add (i32.mul (table.size $t) (i32.const 1000)) (table.size $u))))
    (local.set $r (i32.add (local.get $r)
      (i32.mul (ref.is_null (table.get $u (i32.const 1))) (i32.const 100))))
    (local.set $r (i32.add (local.get $r)
      (i32.mul (ref.is_null (table.get $w (i32.const 0))) (i32.const 10000))))
    (i32.add (local.get $r)
      (i32.add
        (call_indirect $t (type $ii) (local.get $x)
          (i32.rem_u (local.get $x) (i32.add (table.size $t) (i32.const 2))))
        (call_indirect $w (type $ii) (local.get $x)
          (i32.rem_u (i32.shr_u (local.get $x) (i32.const 2)) (i32.const 3))))))
)
""")

# a table that grows to its max, then refuses (-1); the whole table refilled. (Past its
# first min + kTableGrowLimit slots a table widens at run time: WIDE below.)
GROW = assemble(r"""
(module
  (table $t 1 3000 funcref)
  (func $g (result i32) (i32.const 5))
  (elem declare func $g)
  (func (export "grow") (param $n i32) (result i32)
    (local $a i32) (local $b i32)
    (local.set $a (table.grow $t (ref.func $g) (local.get $n)))
    (local.set $b (table.grow $t (ref.null func) (i32.const 0)))
    (table.fill $t (i32.const 0) (ref.func $g) (table.size $t))
    (i32.add (i32.add (local.get $a) (i32.mul (local.get $b) (i32.const 65536)))
             (call_indirect $t (result i32) (i32.sub (table.size $t) (i32.const 1)))))
)
""")

ARGS = [[i] for i in range(130)]
ROUNDS = [ARGS, [[(5 * i + 3) % 130] for i in range(130)], [[(11 * i + 7) % 130] for i in range(130)]]
GROW_ARGS = [[n] for n in (0, 1, 2, 3, 100, 1000, 2998, 2999, 3000, 0xFFFFFFFF, 0x80000000)] * 6


def _oracle(wasm, func, rows):
    m = O.Module(wasm)
    return [O.Instance(m).invoke(func, row) for row in rows]


def _oracle_rounds(wasm, func, rounds):
    m = O.Module(wasm)
    insts = [O.Instance(m) for _ in rounds[0]]
    return [[inst.invoke(func, row) for inst, row in zip(insts, rows)] for rows in rounds]


def test_tables_emulator(built):
    ref = _oracle(TABLES, "run", ARGS)
    codes = {r[0] for r in ref}
    assert len(codes) >= 4, codes     # success plus several distinct table traps
    rets, st, cnt, h = emu_run(TABLES, "run", ARGS, [I32], [I32])
    assert compare(ref, rets, st, cnt, h, [I32]) == []


def test_table_grow_emulator(built):
    ref = _oracle(GROW, "grow", GROW_ARGS)
    rets, st, cnt, h = emu_run(GROW, "grow", GROW_ARGS, [I32], [I32])
    assert compare(ref, rets, st, cnt, h, [I32]) == []


def _gpu_rounds(wasm, func, rounds):
    from wasmedge_amd import batch
    ctx = batch.BatchContext(wasm, len(rounds[0]), device=0)
    out = []
    try:
        for rows in rounds:
            rets, st, cnt = ctx.execute(func, batch.make_values(rows, [I32]), 1)
            ints = batch.ret_ints(rets)
            got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(rows))]
            out.append((got, st, cnt, ctx.memory_hash()))
    finally:
        ctx.close()
    return out


@pytest.mark.gpu
def test_gpu_tables_persist_across_runs(built):
    """Three invocations on the same 130 instances: each lane's tables, sizes and dropped
    element segments carry over between runs as in one reference ModuleInstance."""
    ref = _oracle_rounds(TABLES, "run", ROUNDS)
    for r, (got, st, cnt, h) in enumerate(_gpu_rounds(TABLES, "run", ROUNDS)):
        assert compare(ref[r], got, st, cnt, h, [I32]) == [], "round %d" % r


@pytest.mark.gpu
def test_gpu_table_grow(built):
    ref = _oracle(GROW, "grow", GROW_ARGS)
    got, st, cnt, h = _gpu_rounds(GROW, "grow", [GROW_ARGS])[0]
    assert compare(ref, got, st, cnt, h, [I32]) == []


# Tables widen past their first per-lane capacity (min + kTableGrowLimit): a table.grow
# past it parks the lane, the host relays every lane's tables out wider (hostcall.cpp
# widen_tables) and the grow runs again -- as the reference's Refs vector grows (table.h:
# 59-72) up to the table's max. One big grow per lane, three more of 1500 each, an
# externref table up to its max (past it: -1); the entries written before a relayout
# survive it (call_indirect through slot 0 and through the big grow's last slot).
WIDE = assemble(r"""
(module
  (type $v (func (result i32)))
  (table $t 2 funcref)
  (table $u 1 20000 externref)
  (func $g (type $v) (i32.const 5))
  (func $h (type $v) (i32.const 9))
  (elem declare func $g)
  (elem (table $t) (i32.const 0) func $h)
  (func (export "widen") (param $x i32) (result i32)
    (local $a i32) (local $k i32) (local $s i32) (local $r i32)
    (local.set $a (table.grow $t (ref.func $g) (i32.mul (local.get $x) (i32.const 997))))
    (loop $l
      (local.set $s (i32.add (local.get $s) (table.grow $t (ref.null func) (i32.const 1500))))
      (local.set $k (i32.add (local.get $k) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $k) (i32.const 3))))
    (local.set $s (i32.add (local.get $s)
      (table.grow $u (ref.null extern) (i32.mul (local.get $x) (i32.const 311)))))
    (local.set $r (i32.add (i32.add (local.get $a) (local.get $s))
      (i32.add (i32.mul (table.size $t) (i32.const 7)) (i32.mul (table.size $u) (i32.const 3)))))
    (local.set $r (i32.add (local.get $r)
      (i32.mul (call_indirect $t (type $v) (i32.const 0)) (i32.const 100))))
    (if (local.get $x)
      (then (local.set $r (i32.add (local.get $r)
        (i32.mul (call_indirect $t (type $v) (i32.add (local.get $a) (i32.const 1))) (i32.const 1000))))))
    (i32.add (local.get $r)
      (i32.mul (ref.is_null (table.get $t (i32.sub (table.size $t) (i32.const 1)))) (i32.const 10000))))
)
""")
WIDE_ROUNDS = [[[x] for x in range(130)], [[(7 * x + 3) % 130] for x in range(130)]]


def test_table_widen_emulator(built):
    ref = _oracle_rounds(WIDE, "widen", WIDE_ROUNDS[:1])[0]
    assert max(r[1][0] for r in ref if r[0] == 0) > 4096 * 7   # (past the first capacity)
    rets, st, cnt, h = emu_run(WIDE, "widen", WIDE_ROUNDS[0], [I32], [I32])
    assert compare(ref, rets, st, cnt, h, [I32]) == []


@pytest.mark.gpu
def test_gpu_table_widen(built):
    """Two invocations on the same 130 instances: the second grows the widened tables
    again (and widens them further), entries and sizes carried over."""
    ref = _oracle_rounds(WIDE, "widen", WIDE_ROUNDS)
    for r, (got, st, cnt, h) in enumerate(_gpu_rounds(WIDE, "widen", WIDE_ROUNDS)):
        assert compare(ref[r], got, st, cnt, h, [I32]) == [], "round %d" % r


# Metered: the grow that widens the tables is counted and priced once (the lane parks before
# the step and runs it again), so the limit lands on the same instruction as the oracle's
# whether or not a widening happens there (engine.cpp:1616-1630).
WIDE_LIMITS = list(range(1, 24)) + [40, 1000, 10 ** 6]


def _oracle_metered(wasm, func, rows, limit):
    m = O.Module(wasm)
    return [O.Instance(m, cost_limit=limit).invoke(func, r) for r in rows]


def test_table_widen_metered_emulator(built):
    rows = [[x] for x in (0, 1, 5, 50, 129)]
    for limit in WIDE_LIMITS:
        ref = _oracle_metered(WIDE, "widen", rows, limit)
        rets, st, cnt, h = emu_run(WIDE, "widen", rows, [I32], [I32], cost_limit=limit)
        assert compare(ref, rets, st, cnt, h, [I32]) == [], limit


@pytest.mark.gpu
def test_gpu_table_widen_metered(built):
    from wasmedge_amd import batch
    rows = [[x] for x in range(0, 130, 3)]
    for limit in WIDE_LIMITS:
        if O.Instance(O.Module(WIDE), cost_limit=limit).error:   # instantiation runs out of gas
            with pytest.raises(batch.WasmEdgeError) as e:
                batch.BatchContext(WIDE, len(rows), device=0, cost_limit=limit)
            assert e.value.code == 0x03
            continue
        ref = _oracle_metered(WIDE, "widen", rows, limit)
        ctx = batch.BatchContext(WIDE, len(rows), device=0, cost_limit=limit)
        try:
            rets, st, cnt = ctx.execute("widen", batch.make_values(rows, [I32]), 1)
            ints = batch.ret_ints(rets)
            got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(rows))]
            assert compare(ref, got, st, cnt, ctx.memory_hash(), [I32]) == [], limit
        finally:
            ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("part", [0, 1])
def test_gpu_table_widen_two_shards(built, part):
    """Two shards on one device (multi.cpp): each shard widens its own lanes' tables in its
    own service round; every lane still matches the oracle, over two runs."""
    from wasmedge_amd import batch
    ref = _oracle_rounds(WIDE, "widen", WIDE_ROUNDS)
    ctx = batch.BatchContext(WIDE, len(WIDE_ROUNDS[0]), devices=[0, 0], partition=part)
    try:
        for r, rows in enumerate(WIDE_ROUNDS):
            rets, st, cnt = ctx.execute("widen", batch.make_values(rows, [I32]), 1)
            ints = batch.ret_ints(rets)
            got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(rows))]
            assert compare(ref[r], got, st, cnt, ctx.memory_hash(), [I32]) == [], "round %d" % r
    finally:
        ctx.close()
