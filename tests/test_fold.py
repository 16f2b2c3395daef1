"""Constant folds and fused any_true in compiled runs (jit.cpp plan_folds, DESIGN.md
"Compiled runs"): a splat of an f64 inline constant (0.5, 1, 2, 4 and their negatives) that
only feeds f64x2 add / sub / mul / compares is never materialized (the ops take the
constant), and an any_true that only feeds its run's br_if / br_unless leaves no 0/1 cell.
Both depend on cell liveness, so the module mixes cases that fold with cases that must not:
a constant still live after its run, a splat of a non-inline constant, a subtraction
from the constant (operand order), -0.0 and NaN inputs (whose payload a later store makes
observable), an any_true result used after its branch. Bit-exact against the oracle."""
import ctypes
import os

import pytest

import oracle_py as O
from helpers import compare, gpu_run, oracle_run
from wasmedge_amd.wat import assemble

I32, I64 = 0x7F, 0x7E

FOLD = assemble(r"""
(module
  (memory 1)
  (func (export "run") (param $s i32) (param $n i32) (result i64)
    (local $z v128) (local $w v128) (local $c v128) (local $k v128) (local $i i32) (local $t i32)
    (local.set $z (f64x2.splat (f64.convert_i32_s (local.get $s))))
    (local.set $w (local.get $z))
    (local.set $c (f64x2.replace_lane 1 (f64x2.splat (f64.const 0.25))
                                        (f64.div (f64.convert_i32_s (local.get $s)) (f64.const 7))))
    (block $out (loop $l
      (br_if $out (i32.ge_u (local.get $i) (local.get $n)))
      ;; folded: 4.0 only feeds the compare; the any_true only feeds the branch
      (br_if $out (i32.eqz (v128.any_true (f64x2.le (f64x2.mul (local.get $w) (local.get $w))
                                                    (f64x2.splat (f64.const 4.0))))))
      ;; folded (w's payload is never observed: it only reaches compares): 2.0 * w,
      ;; 0.5 - w (the constant first), w - (-1.0)
      (local.set $w (f64x2.add (f64x2.mul (f64x2.splat (f64.const 2.0)) (local.get $w)) (local.get $c)))
      (local.set $w (f64x2.sub (f64x2.splat (f64.const 0.5)) (local.get $w)))
      (local.set $w (f64x2.sub (local.get $w) (f64x2.splat (f64.const -1.0))))
      ;; not folded: z reaches memory (its payload is observed)
      (local.set $z (f64x2.sub (f64x2.splat (f64.const 0.5)) (f64x2.mul (local.get $z) (local.get $c))))
      ;; not folded: the splat is kept in a local and read after the loop
      (local.set $k (f64x2.splat (f64.const -2.0)))
      (local.set $z (f64x2.mul (local.get $z) (f64x2.mul (local.get $k) (f64x2.splat (f64.const -0.5)))))
      ;; not folded: 3.0 is no inline constant
      (local.set $z (f64x2.add (local.get $z) (f64x2.splat (f64.const 3.0))))
      ;; an any_true kept for later
      (local.set $t (i32.add (local.get $t)
        (v128.any_true (f64x2.gt (local.get $w) (f64x2.splat (f64.const 1.0))))))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br $l)))
    ;; payloads observable: the lanes go to memory
    (v128.store (i32.const 0) (local.get $z))
    (v128.store (i32.const 16) (local.get $k))
    (i64.add (i64.extend_i32_u (i32.add (local.get $t) (i32.mul (local.get $i) (i32.const 1000))))
             (i64.add (i64.load (i32.const 0)) (i64.load (i32.const 8)))))
)
""")


def rows():
    return [[s, n] for s in (-3, -1, 0, 1, 2, 5, 100, -100, 7) for n in (0, 1, 3, 17, 50)]


def test_folds_happen(built, tmp_path):
    """The module really exercises the folds: its compiled code names the constants."""
    from wasmedge_amd import batch
    L = batch.lib()
    L.wb_jit_check.restype = ctypes.c_int
    L.wb_jit_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_uint32]
    dump = tmp_path / "simt.s"
    os.environ["WB_JIT_DUMP_SIMT"] = str(dump)
    try:
        err = ctypes.create_string_buffer(256)
        n = ctypes.c_uint32()
        assert L.wb_jit_check(FOLD, len(FOLD), 7, ctypes.byref(n), err, 256) > 0, err.value
    finally:
        del os.environ["WB_JIT_DUMP_SIMT"]
    src = dump.read_text()
    assert "4.0" in src and "2.0" in src and "0.5" in src


@pytest.mark.gpu
@pytest.mark.parametrize("fold", ["1", "0"])
def test_gpu_folds_match_oracle(built, fold, monkeypatch):
    monkeypatch.setenv("WB_FOLD", fold)
    r = rows()
    ref = oracle_run(O.Module(FOLD), "run", r)
    assert compare(ref, *gpu_run(FOLD, "run", r, [I32, I32], [I64]), [I64], exact=True) == []


# The compare-mask branch (WB_CMPANY): an f64x2 compare feeding a fused any_true
# branch hands its two lane masks to the branch (s_or_b64 of the masks) instead of
# materializing the all-ones cells. br_if and br_unless (eqz) forms, f64x2.ne / lt / eq,
# lanes holding NaN (0/0) and +-inf, so unordered compares take part.
CMPANY = assemble(r"""
(module
  (func (export "run") (param $s i32) (param $n i32) (result i64)
    (local $v v128) (local $i i32) (local $hits i32)
    (local.set $v (f64x2.replace_lane 1 (f64x2.splat (f64.convert_i32_s (local.get $s)))
                    (f64.div (f64.convert_i32_s (local.get $s)) (f64.const 0))))
    (block $out (loop $l
      (br_if $out (i32.ge_u (local.get $i) (local.get $n)))
      (block $a
        (br_if $a (v128.any_true (f64x2.ne (local.get $v) (f64x2.splat (f64.convert_i32_u (local.get $i))))))
        (local.set $hits (i32.add (local.get $hits) (i32.const 1))))
      (block $b
        (br_if $b (i32.eqz (v128.any_true (f64x2.lt (local.get $v) (f64x2.splat (f64.const 2.0))))))
        (local.set $hits (i32.add (local.get $hits) (i32.const 100))))
      (block $c
        (br_if $c (v128.any_true (f64x2.eq (local.get $v) (f64x2.splat (f64.convert_i32_u (local.get $i))))))
        (local.set $hits (i32.add (local.get $hits) (i32.const 10000))))
      (local.set $v (f64x2.add (local.get $v) (f64x2.splat (f64.const 0.5))))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br $l)))
    (i64.extend_i32_u (local.get $hits))))
""")


def cmpany_rows():
    return [[s, n] for s in (-3, -1, 0, 1, 2, 5, -100, 7) for n in (0, 1, 5, 17)]


def test_cmpany_emitted(built, tmp_path):
    """The compiled code of CMPANY ORs the compare's two lane masks into the branch."""
    from wasmedge_amd import batch
    L = batch.lib()
    L.wb_jit_check.restype = ctypes.c_int
    L.wb_jit_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_uint32]
    dump = tmp_path / "simt.s"
    os.environ["WB_JIT_DUMP_SIMT"] = str(dump)
    try:
        err = ctypes.create_string_buffer(256)
        n = ctypes.c_uint32()
        assert L.wb_jit_check(CMPANY, len(CMPANY), 0, ctypes.byref(n), err, 256) > 0, err.value
    finally:
        del os.environ["WB_JIT_DUMP_SIMT"]
    assert "s_or_b64 vcc, vcc, s[68:69]" in dump.read_text()


def test_cmpany_rows_on_oracle():
    """The rows reach both outcomes of each branch (NaN lanes included)."""
    m = O.Module(CMPANY)
    got = {m.run("run", r)[1][0] for r in cmpany_rows()}
    assert len(got) > 8


@pytest.mark.gpu
@pytest.mark.parametrize("cmpany", ["1", "0"])
def test_gpu_cmpany_matches_oracle(built, cmpany, monkeypatch):
    monkeypatch.setenv("WB_CMPANY", cmpany)
    r = cmpany_rows()
    ref = oracle_run(O.Module(CMPANY), "run", r)
    assert compare(ref, *gpu_run(CMPANY, "run", r, [I32, I32], [I64]), [I64], exact=True) == []
