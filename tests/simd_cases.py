"""SIMD128 coverage module for the parity tests: every 0xFD opcode of the reference
(include/common/enum.inc:281-520) applied to per-instance operands, results written to
linear memory (covered by the memory hash) and folded into the return value.

Operands: 16 random vectors from splitmix64(instance id) at 0..255 and 16 fixed
"special" vectors at 256..511 (NaN payloads, signalling NaNs, +-inf, +-0, rounding ties,
trunc_sat range edges, denormals, integer MIN/MAX lane patterns). Instance i uses
vectors A = (i mod 32) and B = (7i + 3) mod 32, so random x special, special x special and
random x random pairs all occur across a batch. Expected values come from the oracle
(the C restatement of the reference, oracle/), compared bit for bit."""
import struct

from wasmedge_amd.opcodes import OPS
from wasmedge_amd.wat import assemble

I32, I64 = 0x7F, 0x7E
OUT = 1024          # result region: 16 bytes per op


def _f32(x):
    return struct.pack("<f", x)


def _f64(x):
    return struct.pack("<d", x)


def _u32(*ws):
    return b"".join(struct.pack("<I", w & 0xFFFFFFFF) for w in ws)


def _u64(*ws):
    return b"".join(struct.pack("<Q", w & 0xFFFFFFFFFFFFFFFF) for w in ws)


SPECIAL = [
    _u32(0x7FC00001, 0xFFA00002, 0x7F800000, 0xFF800000),        # f32 NaNs (q, s), +-inf
    _f32(0.0) + _f32(-0.0) + _f32(1.5) + _f32(-2.5),
    _f32(0.5) + _f32(2.5) + _f32(-0.5) + _f32(3.5),                # nearest ties
    _f32(3e9) + _f32(-3e9) + _f32(2147483648.0) + _f32(4294967296.0),
    _u32(0x00000001, 0x80000010, 0x7F7FFFFF) + _f32(-1.0),         # denormals, FLT_MAX
    _u64(0x7FF8000000000123, 0xFFF0000000000001),                  # f64 NaNs (q, s)
    _u64(0x7FF0000000000000) + _f64(-0.0),
    _f64(2.5) + _f64(-3.5),
    _f64(2147483647.5) + _f64(-2147483648.9),
    _f64(4294967295.9) + _f64(1e300),
    _u64(0x0000000000000001) + _f64(-1.0),
    bytes([0x80, 0x7F, 0xFF, 0x00, 0x01, 0xFE, 0x81, 0x7E, 0x40, 0xC0, 0x3F, 0xBF, 0x10, 0xF0, 0x55, 0xAA]),
    _u32(0x7FFF8000, 0x0000FFFF, 0x80017FFE, 0x00FF0100),
    _u32(0x80000000, 0x7FFFFFFF, 0xFFFFFFFF, 0x00000000),
    _u64(0x8000000000000000, 0x7FFFFFFFFFFFFFFF),
    _f32(1.0) + _f32(2.0) + _u32(0x7F800001, 0x3F800001),
]
assert all(len(v) == 16 for v in SPECIAL)

_NAMES = sorted((n for n, v in OPS.items() if 0xFD00 <= v[0] <= 0xFDFF), key=lambda n: OPS[n][0])


def _classify(n):
    if n in ("v128.any_true",) or n.endswith(".all_true") or n.endswith(".bitmask"):
        return "v:i"
    if n.endswith((".shl", ".shr_s", ".shr_u")):
        return "vi:v"
    if n.endswith(".splat") and not n.startswith("v128.load"):
        return "splat"
    if n == "v128.bitselect":
        return "vvv:v"
    if "lane" in n or n.startswith("v128.load") or n.startswith("v128.store") or \
            n in ("v128.const", "i8x16.shuffle"):
        return "special"
    un = ("v128.not", ".abs", ".neg", ".popcnt", ".ceil", ".floor", ".trunc", ".nearest",
          ".sqrt", "extadd", "extend", "trunc_sat", "convert", "demote", "promote")
    if any(u in n for u in un) and "extmul" not in n:
        return "v:v"
    return "vv:v"


def simd_wat():
    body, k = [], 0
    va = "(v128.load (local.get $a))"
    vb = "(v128.load (local.get $b))"

    def out(expr):
        nonlocal k
        body.append("(v128.store offset=%d (i32.const 0) %s)" % (OUT + 16 * k, expr))
        k += 1

    def out_i32(expr):
        nonlocal k
        body.append("(i32.store offset=%d (i32.const 0) %s)" % (OUT + 16 * k, expr))
        k += 1

    for n in _NAMES:
        c = _classify(n)
        if c == "vv:v":
            out("(%s %s %s)" % (n, va, vb))
            out("(%s %s %s)" % (n, vb, va))
        elif c == "v:v":
            out("(%s %s)" % (n, va))
        elif c == "v:i":
            out_i32("(%s %s)" % (n, va))
            out_i32("(%s (v128.and %s %s))" % (n, va, vb))
        elif c == "vi:v":
            for amt in ("(local.get $s)", "(i32.const 3)", "(i32.const 70)"):
                out("(%s %s %s)" % (n, va, amt))
        elif c == "vvv:v":
            out("(%s %s %s (v128.load offset=16 (local.get $b)))" % (n, va, vb))
        elif c == "splat":
            ty = {"i8x16": "i32", "i16x8": "i32", "i32x4": "i32", "i64x2": "i64",
                  "f32x4": "f32", "f64x2": "f64"}[n.split(".")[0]]
            out("(%s (%s.load offset=4 (local.get $b)))" % (n, ty))
    # lanes: extract every lane of every shape, replace first/last
    shapes = [("i8x16", 16, "i32"), ("i16x8", 8, "i32"), ("i32x4", 4, "i32"),
              ("i64x2", 2, "i64"), ("f32x4", 4, "f32"), ("f64x2", 2, "f64")]
    for sh, nl, ty in shapes:
        exts = [sh + ".extract_lane_s", sh + ".extract_lane_u"] if nl > 4 else [sh + ".extract_lane"]
        for e in exts:
            for lane in range(nl):
                body.append("(%s.store offset=%d (i32.const 0) (%s %d %s))"
                            % (ty, OUT + 16 * k, e, lane, va))
                k += 1
        for lane in (0, nl - 1):
            out("(%s.replace_lane %d %s (%s.load offset=8 (local.get $b)))" % (sh, lane, va, ty))
    # shuffle with indices from both operands
    out("(i8x16.shuffle 0 17 2 19 31 16 5 5 15 14 13 12 30 1 8 24 %s %s)" % (va, vb))
    out("(v128.const i32x4 0x12345678 0x9abcdef0 -1 7)")
    # memory forms at unaligned and aligned addresses
    for ld in ("v128.load", "v128.load8x8_s", "v128.load8x8_u", "v128.load16x4_s",
               "v128.load16x4_u", "v128.load32x2_s", "v128.load32x2_u", "v128.load8_splat",
               "v128.load16_splat", "v128.load32_splat", "v128.load64_splat",
               "v128.load32_zero", "v128.load64_zero"):
        out("(%s offset=3 (local.get $a))" % ld)
        out("(%s offset=8 (local.get $b))" % ld)
    for lanes, w in ((16, 8), (8, 16), (4, 32), (2, 64)):
        for lane in (0, lanes - 1):
            out("(v128.load%d_lane offset=1 %d (local.get $a) %s)" % (w, lane, vb))
            body.append("(v128.store%d_lane offset=%d %d (i32.const 0) %s)"
                        % (w, OUT + 16 * k + 3, lane, va))
            k += 1
    nout = k
    wat = r"""
(module
  (memory 1)
  (data (i32.const 256) "%s")
  (func $fill (param $iid i32)
    (local $i i32) (local $x i64)
    (local.set $x (i64.xor (i64.extend_i32_u (local.get $iid)) (i64.const 0x5EED)))
    (loop $l
      (local.set $x (i64.add (local.get $x) (i64.const 0x9E3779B97F4A7C15)))
      (i64.store (local.get $i)
        (call $mix (local.get $x)))
      (local.set $i (i32.add (local.get $i) (i32.const 8)))
      (br_if $l (i32.lt_u (local.get $i) (i32.const 256)))))
  (func $mix (param $z i64) (result i64)
    (local.set $z (i64.mul (i64.xor (local.get $z) (i64.shr_u (local.get $z) (i64.const 30)))
                           (i64.const 0xBF58476D1CE4E5B9)))
    (local.set $z (i64.mul (i64.xor (local.get $z) (i64.shr_u (local.get $z) (i64.const 27)))
                           (i64.const 0x94D049BB133111EB)))
    (i64.xor (local.get $z) (i64.shr_u (local.get $z) (i64.const 31))))
  (func (export "simd") (param $iid i32) (result i64)
    (local $a i32) (local $b i32) (local $s i32) (local $i i32) (local $acc i64)
    (call $fill (local.get $iid))
    (local.set $a (i32.shl (i32.rem_u (local.get $iid) (i32.const 32)) (i32.const 4)))
    (local.set $b (i32.shl (i32.rem_u (i32.add (i32.mul (local.get $iid) (i32.const 7))
                                               (i32.const 3)) (i32.const 32)) (i32.const 4)))
    (if (i32.eq (local.get $b) (i32.const 496)) (then (local.set $b (i32.const 480))))
    (local.set $s (i32.rem_u (i32.mul (local.get $iid) (i32.const 13)) (i32.const 70)))
    %s
    (loop $l
      (local.set $acc (i64.add (i64.rotl (local.get $acc) (i64.const 7))
                               (i64.load offset=%d (local.get $i))))
      (local.set $i (i32.add (local.get $i) (i32.const 8)))
      (br_if $l (i32.lt_u (local.get $i) (i32.const %d))))
    (local.get $acc))
  (func (export "lane_oob") (param $addr i32) (param $w i32) (result i32)
    (local $v v128)
    (local.set $v (v128.const i64x2 0x0102030405060708 0x1112131415161718))
    (block $b3 (block $b2 (block $b1 (block $b0
      (br_table $b0 $b1 $b2 $b3 (local.get $w)))
      (local.set $v (v128.load8_lane 3 (local.get $addr) (local.get $v))) (br $b3))
      (local.set $v (v128.load64_lane offset=2 1 (local.get $addr) (local.get $v))) (br $b3))
      (v128.store32_lane 2 (local.get $addr) (local.get $v)) (br $b3))
    (v128.store16_lane offset=4 7 (local.get $addr) (local.get $v))
    (i32x4.extract_lane 1 (local.get $v)))
)
""" % ("".join("\\%02x" % b for b in b"".join(SPECIAL)), "\n    ".join(body), OUT, nout * 16)
    return wat, nout


def simd_wasm():
    return assemble(simd_wat()[0])


def ops_covered():
    """Every 0xFD opcode the module's text names (asserted complete by the tests)."""
    wat = simd_wat()[0]
    return {n for n in _NAMES if n in wat}


def all_simd_ops():
    return set(_NAMES)
