"""NaN payload liveness (jit.cpp nan_observable): the compiled runs give an f32/f64 add,
sub or mul NaN result the reference's x86 payload only where the payload can be observed
-- returned, stored, kept in a global, passed on, or read as bits. Results that only ever
reach a float compare (the Mandelbrot iteration) need no fix.

CPU: the analysis removes every fix from C5's module and keeps the fixes of a module that
returns, stores or reinterprets its NaNs. GPU: such a module, with NaNs made fresh
(inf - inf, 0 * inf) and propagated from parameters, is bit-exact against the oracle
(returned payloads, memory hash, globals through a getter) with the analysis on and off."""
import ctypes
import math
import os
import struct

import pytest

import oracle_py as O
from helpers import compare, gpu_run, oracle_run
from wasmedge_amd import workloads as W
from wasmedge_amd.wat import assemble

I32, I64, F64 = 0x7F, 0x7E, 0x7C
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

NAN_WAT = r"""
(module
  (memory 1)
  (global $g (mut f64) (f64.const 0))
  ;; x, y per instance; k picks the path. Fresh NaNs: inf - inf, 0 * inf; propagated NaNs:
  ;; a NaN x with its own payload.
  (func (export "f") (param $x f64) (param $y f64) (param $k i32) (result i64)
    (local $a f64) (local $b f64) (local $v v128) (local $n i32) (local $acc i64)
    (local $c f64) (local $d f64)
    (local.set $a (f64.sub (f64.mul (local.get $x) (local.get $y)) (local.get $y)))
    (local.set $b (f64.add (local.get $a) (local.get $x)))
    ;; a loop whose values are later returned, stored or read as bits (its fixes stay)
    (block $done
      (loop $l
        (local.set $a (f64.mul (local.get $a) (local.get $a)))
        (local.set $b (f64.sub (local.get $b) (local.get $a)))
        (local.set $n (i32.add (local.get $n) (i32.const 1)))
        (br_if $done (f64.gt (local.get $b) (f64.const 1e300)))
        (br_if $l (i32.lt_u (local.get $n) (i32.const 6)))))
    ;; a second loop whose values only ever reach a compare (its fixes may go)
    (local.set $c (f64.mul (local.get $x) (local.get $y)))
    (local.set $d (f64.sub (local.get $c) (local.get $y)))
    (local.set $n (i32.const 0))
    (block $done2
      (loop $l2
        (local.set $c (f64.mul (local.get $c) (local.get $d)))
        (local.set $d (f64.add (local.get $d) (local.get $c)))
        (local.set $n (i32.add (local.get $n) (i32.const 1)))
        (br_if $done2 (f64.ge (local.get $c) (local.get $d)))
        (br_if $l2 (i32.lt_u (local.get $n) (i32.const 5)))))
    (local.set $v (f64x2.mul (f64x2.splat (local.get $x)) (f64x2.splat (local.get $y))))
    (local.set $v (f64x2.sub (local.get $v) (f64x2.splat (local.get $y))))
    (if (i32.eq (local.get $k) (i32.const 0))   ;; returned as bits
      (then (return (i64.reinterpret_f64 (local.get $b)))))
    (if (i32.eq (local.get $k) (i32.const 1))   ;; stored
      (then (f64.store (i32.const 8) (local.get $a)) (return (i64.const 1))))
    (if (i32.eq (local.get $k) (i32.const 2))   ;; kept in a global
      (then (global.set $g (f64.mul (local.get $b) (local.get $y))) (return (i64.const 2))))
    (if (i32.eq (local.get $k) (i32.const 3))   ;; v128 lanes stored
      (then (v128.store (i32.const 16) (local.get $v)) (return (i64.const 3))))
    (if (i32.eq (local.get $k) (i32.const 4))   ;; bits compared as an integer
      (then (return (i64.extend_i32_u (i64.eq (i64.reinterpret_f64 (local.get $a))
                                                (i64.const 0xfff8000000000000))))))
    ;; only compared: nothing observable
    (i64.extend_i32_u (f64.lt (local.get $a) (local.get $b))))
  (func (export "g") (result i64) (i64.reinterpret_f64 (global.get $g))))
"""


def f64bits(v):
    return struct.unpack("<Q", struct.pack("<d", v))[0]


QNAN_PAYLOAD = 0x7FF4000000001234   # a signalling-bit-clear NaN with a payload


def rows():
    xs = [1.5, math.inf, 0.0, -math.inf, QNAN_PAYLOAD, 3.0, -0.0, 1e200]
    ys = [2.0, math.inf, math.inf, 0.0, 1.0, QNAN_PAYLOAD | (1 << 63), -math.inf, 1e200]
    out = []
    for i in range(48):
        x, y = xs[i % len(xs)], ys[(i // len(xs)) % len(ys)]
        bx = x if isinstance(x, int) else f64bits(x)
        by = y if isinstance(y, int) else f64bits(y)
        out.append([bx, by, i % 6])
    return out


def _check_lib():
    L = ctypes.CDLL(os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch.so"))
    L.wb_jit_check.restype = ctypes.c_int
    L.wb_jit_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32]
    return L


def _nan_checks(wasm, monkeypatch, tmp_path, on):
    """v_cmp_u (a NaN fix's test) in the compiled SIMT code of `wasm`"""
    dump = tmp_path / ("simt_%d.s" % on)
    monkeypatch.setenv("WB_JIT_DUMP_SIMT", str(dump))
    monkeypatch.setenv("WB_NANOBS", "1" if on else "0")
    err = ctypes.create_string_buffer(4096)
    assert _check_lib().wb_jit_check(wasm, len(wasm), 0, None, err, 4096) >= 0, err.value
    return dump.read_text().count("v_cmp_u_f")


def test_analysis_drops_unobserved_fixes(built, monkeypatch, tmp_path):
    mandel = W.mandel_wasm()
    assert _nan_checks(mandel, monkeypatch, tmp_path, False) > 0
    assert _nan_checks(mandel, monkeypatch, tmp_path, True) == 0
    m = assemble(NAN_WAT)
    off, on = _nan_checks(m, monkeypatch, tmp_path, False), _nan_checks(m, monkeypatch, tmp_path, True)
    assert 0 < on < off   # the loop's fixes go, the observed results' stay


@pytest.mark.gpu
@pytest.mark.parametrize("nanobs", ["1", "0"])
def test_gpu_nan_payloads_observed_paths(built, monkeypatch, nanobs):
    monkeypatch.setenv("WB_NANOBS", nanobs)
    wasm = assemble(NAN_WAT)
    rs = rows()
    ref = oracle_run(O.Module(wasm), "f", rs)
    got = gpu_run(wasm, "f", rs, [F64, F64, I32], [I64])
    assert compare(ref, *got, [I64], exact=True) == []
    # the global, read back through a getter on the same instances (state persists)
    from wasmedge_amd import batch
    ctx = batch.BatchContext(wasm, len(rs), device=0)
    try:
        ctx.execute("f", batch.make_values(rs, [F64, F64, I32]), 1)
        rets, st, _ = ctx.execute("g", batch.make_values([[] for _ in rs], []), 1)
        vals = batch.ret_ints(rets)
    finally:
        ctx.close()
    for i, r in enumerate(rs):
        inst = O.Instance(O.Module(wasm))
        inst.invoke("f", r)
        code, v, _, _ = inst.invoke("g", [])
        assert int(st[i]) == code == 0 and int(vals[i][0]) == v[0], i
