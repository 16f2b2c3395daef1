"""Recursive modules under SIMT scheduling (jit.cpp sched_block, DESIGN.md "SIMT
scheduling"): a module whose functions can reach themselves picks the next group by
call-stack height first, and its split branches go through that pick. The pick only
reorders which lanes run when, so every lane's result, count and memory must equal the
oracle's whatever the policy: lanes of mixed recursion depths through direct, mutual,
three-way and table-driven recursion, some past the LDS part of the call stack (where the
C++ step holds their frames and a compiled return meets them: its record reads ~0 and the
group leaves), with the pick on and off (WB_DEPTH=0)."""
import ctypes
import os

import pytest

import oracle_py as O
from helpers import compare, gpu_run, oracle_run
from wasmedge_amd.wat import assemble

I32, I64 = 0x7F, 0x7E

REC = assemble(r"""
(module
  (type $t1 (func (param i32) (result i32)))
  (table 2 funcref)
  (elem (i32.const 0) $viat $dec)
  (memory 1)
  ;; three call sites per frame
  (func $tri (param $n i32) (result i32)
    (if (result i32) (i32.lt_s (local.get $n) (i32.const 3))
      (then (i32.add (local.get $n) (i32.const 1)))
      (else (i32.add (call $tri (i32.sub (local.get $n) (i32.const 1)))
                     (i32.xor (call $tri (i32.sub (local.get $n) (i32.const 2)))
                              (call $tri (i32.sub (local.get $n) (i32.const 3))))))))
  ;; mutual recursion with a store per frame (deep lanes pass the LDS part of the stack)
  (func $even (param $n i32) (result i32)
    (i32.store (i32.and (i32.shl (local.get $n) (i32.const 2)) (i32.const 4092)) (local.get $n))
    (if (result i32) (i32.eqz (local.get $n))
      (then (i32.const 1))
      (else (i32.add (i32.const 2) (call $odd (i32.sub (local.get $n) (i32.const 1)))))))
  (func $odd (param $n i32) (result i32) (local $k i32)
    (local.set $k (i32.mul (local.get $n) (i32.const 7)))
    (if (result i32) (i32.eqz (local.get $n))
      (then (i32.const 0))
      (else (i32.xor (local.get $k) (call $even (i32.sub (local.get $n) (i32.const 1)))))))
  ;; Ackermann A(m, n) for small m: deep, irregular call trees
  (func $ack (param $m i32) (param $n i32) (result i32)
    (if (result i32) (i32.eqz (local.get $m))
      (then (i32.add (local.get $n) (i32.const 1)))
      (else (if (result i32) (i32.eqz (local.get $n))
        (then (call $ack (i32.sub (local.get $m) (i32.const 1)) (i32.const 1)))
        (else (call $ack (i32.sub (local.get $m) (i32.const 1))
                         (call $ack (local.get $m) (i32.sub (local.get $n) (i32.const 1)))))))))
  ;; recursion through the table, with a loop in each frame
  (func $viat (param $n i32) (result i32) (local $i i32) (local $s i32)
    (block $out (loop $l
      (br_if $out (i32.ge_u (local.get $i) (i32.and (local.get $n) (i32.const 3))))
      (local.set $s (i32.add (local.get $s) (i32.mul (local.get $i) (local.get $n))))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br $l)))
    (if (result i32) (i32.le_u (local.get $n) (i32.const 1))
      (then (local.get $s))
      (else (i32.add (local.get $s)
        (call_indirect (type $t1) (i32.sub (local.get $n) (i32.const 1))
                                  (i32.and (local.get $n) (i32.const 1)))))))
  (func $dec (param $n i32) (result i32)
    (if (result i32) (i32.eqz (local.get $n))
      (then (i32.const 0))
      (else (i32.add (i32.const 1) (call $viat (i32.sub (local.get $n) (i32.const 1)))))))
  (func (export "run") (param $which i32) (param $n i32) (result i32)
    (if (result i32) (i32.eq (local.get $which) (i32.const 0))
      (then (call $tri (local.get $n)))
      (else (if (result i32) (i32.eq (local.get $which) (i32.const 1))
        (then (call $even (local.get $n)))
        (else (if (result i32) (i32.eq (local.get $which) (i32.const 2))
          (then (call $ack (i32.and (local.get $n) (i32.const 3)) (i32.shr_u (local.get $n) (i32.const 2))))
          (else (call $viat (local.get $n)))))))))
)
""")

# straight-line and loop code only: no recursion, the pc-only pick stays
FLAT = assemble(r"""
(module
  (func $sq (param i32) (result i32) (i32.mul (local.get 0) (local.get 0)))
  (func (export "run") (param $n i32) (result i32) (local $i i32) (local $s i32)
    (block $o (loop $l
      (br_if $o (i32.ge_u (local.get $i) (local.get $n)))
      (local.set $s (i32.add (local.get $s) (call $sq (local.get $i))))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br $l)))
    (local.get $s)))
""")


def rows():
    out = []
    for k in range(256):
        w = k % 4
        if w == 0:
            n = 3 + (k * 7) % 16            # tri(3..18)
        elif w == 1:
            n = [0, 1, 5, 40, 300, 2500, 5000][k % 7]   # mutual, up to 5,000 frames
        elif w == 2:
            n = (k * 13) % 28               # ack(m <= 3, n <= 6)
        else:
            n = 2 + (k * 5) % 60            # through the table
        out.append([w, n])
    return out


def test_recursion_detected(built):
    """wb_trip_choice's sibling hook: which modules count as recursive (a direct-call cycle
    or any indirect call), which decides the depth-keyed pick."""
    from wasmedge_amd import batch
    L = batch.lib()
    L.wb_recursive.restype = ctypes.c_int
    L.wb_recursive.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
    fib = open(os.path.join(os.path.dirname(__file__), "golden", "fibonacci.wasm"), "rb").read()
    assert L.wb_recursive(REC, len(REC)) == 1
    assert L.wb_recursive(fib, len(fib)) == 1
    assert L.wb_recursive(FLAT, len(FLAT)) == 0


def test_oracle_sanity():
    m = O.Module(REC)
    assert m.run("run", [2, 2 + 4 * 3])[1] == [9]        # A(2, 3) = 2*3 + 3


@pytest.mark.gpu
@pytest.mark.parametrize("depth", ["1", "0"])
def test_gpu_recursive_matches_oracle(built, depth, monkeypatch):
    """256 lanes of mixed recursion (four shapes, depths from 0 to 5,000 frames) bit-exact
    against the oracle: results, counts, memory; with the depth-keyed pick and without."""
    monkeypatch.setenv("WB_DEPTH", depth)
    r = rows()
    ref = oracle_run(O.Module(REC), "run", r)
    got = gpu_run(REC, "run", r, [I32, I32], [I32], call_stack_cells=1 << 16)
    assert compare(ref, *got, [I32]) == []


@pytest.mark.gpu
def test_gpu_flat_matches_oracle(built):
    r = [[n] for n in range(0, 640, 5)]
    ref = oracle_run(O.Module(FLAT), "run", r)
    assert compare(ref, *gpu_run(FLAT, "run", r, [I32], [I32]), [I32]) == []
