"""Limits of this build that the reference does not have (VERDICT r2 "what's missing" 6),
pinned at their boundary, and one that is gone:

* count corrections: a branch's taken-count correction is a 16-bit field. Folded
  instructions pending before a label now go into NOP_CNT carriers first (frontend.cpp
  spill_pending), so the correction stays within [-255, 0] however many precede the
  label. Before, 40,000 `nop`s in front of a loop gave a backward branch a correction of
  -40,000, silently truncated (counts off by 65,536 per taken branch), and in front of a
  block end a "tcnt overflow" rejection. The reference counts every `nop`
  (engine.cpp:1618-1631), so this is counting parity, exact against the oracle.
* segment counts: data segments and element segments of any number, each dropped
  per instance (a bit per segment in the instance state; round 3 refused more than 32
  data segments with `data.drop` and more than 32 element segments in a table-mutating
  module). Modules with 70 segments of each kind -- passive and active ones, memory.init /
  table.init from segments in every mask word, data.drop / elem.drop on some lanes, state
  kept across invocations -- run bit-exact against the oracle (the reference has no limit,
  lib/executor/instantiate/data.cpp, elem.cpp).
"""
import pytest

from wasmedge_amd.wat import assemble
from helpers import emu_run, oracle_run, compare

import oracle_py as O

I32 = 0x7F


def nops_module(n):
    nops = " ".join(["nop"] * n)
    return assemble(r"""
(module
  (func (export "f") (param $x i32) (result i32)
    (local $k i32)
    %s
    (loop $l
      (local.set $k (i32.add (local.get $k) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $k) (local.get $x))))
    (block $b
      (local.set $k (i32.add (local.get $k) (i32.const 100)))
      (br_if $b (i32.and (local.get $x) (i32.const 1)))
      %s
      (local.set $k (i32.add (local.get $k) (i32.const 1000))))
    (local.get $k)))
""" % (nops, nops))


def data_module(nseg):
    """nseg data segments: every 5th active (at 1024 + k), the rest passive; f(x) inits
    bytes from segments 2, 33, nseg-4 (passive) and nseg-5 (active: dropped at
    instantiation, so a 1-byte init traps 0x88 when x & 4), drops 33 and nseg-4 when x & 1."""
    def seg(k):
        return ('  (data $d%d (i32.const %d) "\\%02x")' % (k, 1024 + k, k) if k % 5 == 0
                else '  (data $d%d "\\%02x\\%02x")' % (k, k, k + 1))
    segs = "\n".join(seg(k) for k in range(nseg))
    act = nseg - 5 - (nseg - 5) % 5
    return assemble(r"""
(module
  (memory 1)
%s
  (func (export "f") (param $x i32) (result i32)
    (memory.init $d2 (i32.const 8) (i32.const 0) (i32.const 1))
    (memory.init $d33 (i32.const 9) (i32.const 1) (i32.const 1))
    (memory.init $d%d (i32.const 10) (i32.const 0) (i32.const 2))
    (memory.init $d%d (i32.const 12) (i32.const 0) (i32.const 0))
    (if (i32.and (local.get $x) (i32.const 4))
      (then (memory.init $d%d (i32.const 12) (i32.const 0) (i32.const 1))))
    (if (i32.and (local.get $x) (i32.const 1)) (then (data.drop $d33) (data.drop $d%d)))
    (i32.add (i32.load (i32.const 8)) (i32.load8_u (i32.const %d)))))
""" % (segs, nseg - 4, act, act, nseg - 4, 1024 + act))


def elem_module(nseg):
    """nseg element segments (every 7th active into table $t at 1, the rest passive);
    f(x) table.inits from segments 36 and nseg-1, drops them when x & 1."""
    segs = "\n".join(("  (elem $e%d (table $t) (i32.const 1) func $g)" % k) if k % 7 == 0
                     else ("  (elem $e%d func %s)" % (k, "$g" if k % 2 else "$h")) for k in range(nseg))
    return assemble(r"""
(module
  (table $t 4 funcref)
  (type $v (func (result i32)))
  (func $g (result i32) (i32.const 7))
  (func $h (result i32) (i32.const 11))
%s
  (func (export "f") (param $x i32) (result i32)
    (table.init $t $e36 (i32.const 0) (i32.const 0) (i32.const 1))
    (table.init $t $e%d (i32.const 2) (i32.const 0) (i32.const 1))
    (if (i32.and (local.get $x) (i32.const 1)) (then (elem.drop $e36) (elem.drop $e%d)))
    (i32.add (call_indirect (type $v) (i32.const 0))
             (i32.mul (i32.const 100) (call_indirect (type $v) (i32.const 2))))))
""" % (segs, nseg - 1, nseg - 1))


ROWS = [[x] for x in (0, 1, 2, 5, 6)]


@pytest.mark.parametrize("n", [300, 40000])
def test_long_folded_prefix_counts_emulator(built, n):
    wasm = nops_module(n)
    ref = oracle_run(O.Module(wasm), "f", ROWS)
    got = emu_run(wasm, "f", ROWS, [I32], [I32])
    assert compare(ref, *got, [I32]) == []


ROWS_SEG = [[x] for x in (0, 1, 2, 3, 4, 5, 6, 7)]


@pytest.mark.parametrize("make", [data_module, elem_module])
@pytest.mark.parametrize("nseg", [40, 70])
def test_many_segments_emulator(built, make, nseg):
    wasm = make(nseg)
    ref = oracle_run(O.Module(wasm), "f", ROWS_SEG)
    assert {r[0] for r in ref} <= {0, 0x88}
    assert compare(ref, *emu_run(wasm, "f", ROWS_SEG, [I32], [I32]), [I32]) == []


@pytest.mark.gpu
def test_gpu_limits(built):
    from helpers import gpu_run
    for wasm in (nops_module(40000), data_module(40), elem_module(40)):
        ref = oracle_run(O.Module(wasm), "f", ROWS)
        assert compare(ref, *gpu_run(wasm, "f", ROWS, [I32], [I32]), [I32]) == []


@pytest.mark.gpu
@pytest.mark.parametrize("make", [data_module, elem_module])
def test_gpu_many_segments(built, make):
    """70 segments: masks past the first word, on 130 lanes (three waves), invoked twice on
    the same instances -- the second call sees the first call's drops -- against an oracle
    instance kept across the two calls."""
    from wasmedge_amd import batch
    wasm = make(70)
    rows = [[x % 8] for x in range(130)]
    m = O.Module(wasm)
    want = []
    for r in rows:
        inst = O.Instance(m)
        want.append([inst.invoke("f", r)[:2], inst.invoke("f", r)[:2]])
    ctx = batch.BatchContext(wasm, len(rows), device=0)
    try:
        got = []
        for rep in range(2):
            rets, st, cnt = ctx.execute("f", batch.make_values(rows, [I32]), 1)
            got.append([(int(st[i]), [int(batch.ret_ints(rets)[i][0])] if st[i] == 0 else [])
                        for i in range(len(rows))])
        for i in range(len(rows)):
            for rep in range(2):
                code, vals = want[i][rep]
                assert got[rep][i] == (code, list(vals) if code == 0 else []), (i, rep)
    finally:
        ctx.close()
