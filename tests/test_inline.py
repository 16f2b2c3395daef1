"""Inlined calls in the compiled runs (jit.cpp "Inlined call", DESIGN.md "Compiled runs").

A call to a leaf function that is one compiled run ending in its return runs inside the
caller's code, the callee's cells shifted above the caller's live cells; a leave inside the
callee (a misaligned or out-of-bounds access, a NaN result leaves nothing) first makes the
call real (spill, return record, cells back to the frame base) so that the C++ step meets
the reference layout. These modules call such a leaf from a loop with per-lane addresses
that are sometimes misaligned (the C++ step performs the access) and sometimes past the one
page of memory on the lanes whose address mask reaches past it (0x88 at the exact
instruction inside the callee), with the caller's live
cells at both parities (only even shifts are inlined), and check every lane against the
oracle bit for bit with inlining on and off."""
import ctypes
import os

import pytest

import oracle_py as O
from helpers import compare, gpu_run
from wasmedge_amd.wat import assemble

I32 = 0x7F
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS = [[(i * 2654435761 + 977) & 0xFFFFFFFF] for i in range(192)]


def leaf_module(extra_locals):
    locs = " ".join("(local $e%d i32)" % k for k in range(extra_locals))
    uses = " ".join("(local.set $e%d (i32.add (local.get $e%d) (local.get $i)))" % (k, k)
                    for k in range(extra_locals))
    fold = "".join("(i32.xor (local.get $e%d) " % k for k in range(extra_locals))
    return assemble(r"""
(module
  (memory 1)
  (func $leaf (param $p i32) (param $q i32) (result i32)
    (local $t i32) (local $u i32)
    (local.set $t (i32.load offset=4 (local.get $p)))
    (local.set $u (i32.rotl (i32.add (local.get $t) (local.get $q)) (i32.const 7)))
    (i32.store (local.get $q) (i32.xor (local.get $u) (local.get $p)))
    (i32.add (local.get $u) (i32.load16_u offset=2 (local.get $q))))
  (func (export "run") (param $s i32) (result i32)
    (local $i i32) (local $acc i32) %s
    (loop $l
      %s
      (local.set $acc (i32.add (local.get $acc)
        (call $leaf
          (i32.and (i32.mul (local.get $s) (i32.add (local.get $i) (i32.const 1)))
                   (i32.or (i32.const 0xFFFF) (i32.and (local.get $s) (i32.const 0x10000))))
          (i32.and (i32.add (local.get $s) (i32.mul (local.get $i) (i32.const 40503))) (i32.const 0x3FFF)))))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $i) (i32.const 24))))
    %s (local.get $acc) %s))
""" % (locs, uses, fold, ")" * extra_locals))


def _inlined(wasm):
    """how many call sites the compiled SIMT code inlines (wb_jit_check's dump)"""
    L = ctypes.CDLL(os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch.so"))
    L.wb_jit_check.restype = ctypes.c_int
    L.wb_jit_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_uint32]
    path = "/tmp/wb_inline_%d.s" % os.getpid()
    os.environ["WB_JIT_DUMP_SIMT"] = path
    try:
        err = ctypes.create_string_buffer(4096)
        assert L.wb_jit_check(wasm, len(wasm), 0, None, err, 4096) >= 0, err.value
        return open(path).read().count('"Lii')
    finally:
        os.environ.pop("WB_JIT_DUMP_SIMT", None)


def test_inlined_call_sites(built):
    """the generator gives both parities of the caller's live cells; even ones inline"""
    got = [_inlined(leaf_module(k)) for k in range(4)]
    assert any(got) and not all(got), got


def test_leaf_modules_trap_and_succeed():
    codes = set()
    for k in range(4):
        m = O.Module(leaf_module(k))
        codes |= {m.run("run", r)[0] for r in ROWS}
    assert 0 in codes and 0x88 in codes


@pytest.mark.gpu
@pytest.mark.parametrize("inline", ["1", "0"])
def test_gpu_inlined_calls_bit_exact(built, monkeypatch, inline):
    monkeypatch.setenv("WB_INLINE", inline)
    for k in range(4):
        wasm = leaf_module(k)
        ref = [O.Module(wasm).run("run", r) for r in ROWS]
        rets, st, cnt, h = gpu_run(wasm, "run", ROWS, [I32], [I32])
        assert compare(ref, rets, st, cnt, h, [I32], exact=True) == [], k
