"""Limits of this build that the reference does not have (VERDICT r2 "what's missing" 6),
pinned at their boundary, and one that is gone:

* count corrections: a branch's taken-count correction is a 16-bit field. Folded
  instructions pending before a label now go into NOP_CNT carriers first (frontend.cpp
  spill_pending), so the correction stays within [-255, 0] however many precede the
  label. Before, 40,000 `nop`s in front of a loop gave a backward branch a correction of
  -40,000, silently truncated (counts off by 65,536 per taken branch), and in front of a
  block end a "tcnt overflow" rejection. The reference counts every `nop`
  (engine.cpp:1618-1631), so this is counting parity, exact against the oracle.
* at most 32 data segments when the module uses `data.drop` (the dropped set is one
  32-bit word per instance), and at most 32 element segments in a module that mutates
  its tables (per-lane tables, frontend.cpp). Both fail BatchCreate with 0x02 and a
  message; one fewer is accepted and runs bit-exact. The reference has no such limit
  (DESIGN.md "Module subset").
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
    segs = "\n".join('  (data $d%d "\\%02x")' % (k, k) for k in range(nseg))
    return assemble(r"""
(module
  (memory 1)
%s
  (func (export "f") (param $x i32) (result i32)
    (memory.init $d%d (i32.const 8) (i32.const 0) (i32.const 1))
    (if (local.get $x) (then (data.drop $d%d)))
    (i32.load8_u (i32.const 8))))
""" % (segs, nseg - 1, nseg - 1))


def elem_module(nseg):
    segs = "\n".join("  (elem $e%d func $g)" % k for k in range(nseg))
    return assemble(r"""
(module
  (table $t 2 funcref)
  (type $v (func (result i32)))
  (func $g (result i32) (i32.const 7))
%s
  (func (export "f") (param $x i32) (result i32)
    (table.init $t $e%d (i32.const 0) (i32.const 0) (i32.const 1))
    (if (local.get $x) (then (elem.drop $e%d)))
    (call_indirect (type $v) (i32.const 0))))
""" % (segs, nseg - 1, nseg - 1))


ROWS = [[x] for x in (0, 1, 2, 5, 6)]


@pytest.mark.parametrize("n", [300, 40000])
def test_long_folded_prefix_counts_emulator(built, n):
    wasm = nops_module(n)
    ref = oracle_run(O.Module(wasm), "f", ROWS)
    got = emu_run(wasm, "f", ROWS, [I32], [I32])
    assert compare(ref, *got, [I32]) == []


@pytest.mark.parametrize("kind,make", [("data", data_module), ("element", elem_module)])
def test_segment_limit_boundary_emulator(built, kind, make):
    ok = make(32)
    ref = oracle_run(O.Module(ok), "f", ROWS)
    assert compare(ref, *emu_run(ok, "f", ROWS, [I32], [I32]), [I32]) == []
    # the oracle (the reference's behaviour) runs 33; this build refuses it at lowering
    bad = make(33)
    assert all(r[0] == 0 for r in oracle_run(O.Module(bad), "f", ROWS))
    with pytest.raises(RuntimeError, match="0x2: more than 32 %s segments" % kind):
        emu_run(bad, "f", ROWS, [I32], [I32])


@pytest.mark.gpu
def test_gpu_limits(built):
    from helpers import gpu_run
    from wasmedge_amd import batch
    for wasm in (nops_module(40000), data_module(32), elem_module(32)):
        ref = oracle_run(O.Module(wasm), "f", ROWS)
        assert compare(ref, *gpu_run(wasm, "f", ROWS, [I32], [I32]), [I32]) == []
    for make in (data_module, elem_module):
        with pytest.raises(RuntimeError):
            batch.BatchContext(make(33), 4, device=0)
