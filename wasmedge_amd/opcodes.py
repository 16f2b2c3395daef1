"""WebAssembly opcode table (text name -> binary encoding + immediate kind).

The numbering is the final WebAssembly 1.0 + sign-ext + sat-trunc + bulk-memory +
reference-types + SIMD128 numbering, which is the numbering the reference decodes
(`include/common/enum.inc:54-541`, `lib/loader/ast/instruction.cpp:14-32`: one byte, or a
0xFC/0xFD prefix byte followed by a LEB128 u32).  This table is the build's own; it is used
by the WAT assembler (`wat.py`) that authors the config modules, because no wasm-producing
toolchain exists in this image.
"""

# immediate kinds
NONE, BLOCK, LABEL, BRTABLE, FUNC, CALLIND, LOCAL, GLOBAL, MEM, I32, I64, F32, F64, \
    MEMIDX, TABLE, SELECTT, REFNULL, V128, LANE, SHUFFLE, MEMLANE, TWOIDX, DATA, ELEM, \
    MEMMEM = range(25)

OPS = {}


def _op(name, code, imm=NONE, align=0):
    OPS[name] = (code, imm, align)


for _n, _c, _i in [
    ("unreachable", 0x00, NONE), ("nop", 0x01, NONE), ("block", 0x02, BLOCK),
    ("loop", 0x03, BLOCK), ("if", 0x04, BLOCK), ("else", 0x05, NONE), ("end", 0x0B, NONE),
    ("br", 0x0C, LABEL), ("br_if", 0x0D, LABEL), ("br_table", 0x0E, BRTABLE),
    ("return", 0x0F, NONE), ("call", 0x10, FUNC), ("call_indirect", 0x11, CALLIND),
    ("return_call", 0x12, FUNC), ("return_call_indirect", 0x13, CALLIND),
    ("drop", 0x1A, NONE), ("select", 0x1B, SELECTT),
    ("local.get", 0x20, LOCAL), ("local.set", 0x21, LOCAL), ("local.tee", 0x22, LOCAL),
    ("global.get", 0x23, GLOBAL), ("global.set", 0x24, GLOBAL),
    ("table.get", 0x25, TABLE), ("table.set", 0x26, TABLE),
    ("memory.size", 0x3F, MEMIDX), ("memory.grow", 0x40, MEMIDX),
    ("i32.const", 0x41, I32), ("i64.const", 0x42, I64), ("f32.const", 0x43, F32),
    ("f64.const", 0x44, F64),
    ("ref.null", 0xD0, REFNULL), ("ref.is_null", 0xD1, NONE), ("ref.func", 0xD2, FUNC),
]:
    _op(_n, _c, _i)

for _n, _c, _a in [
    ("i32.load", 0x28, 2), ("i64.load", 0x29, 3), ("f32.load", 0x2A, 2), ("f64.load", 0x2B, 3),
    ("i32.load8_s", 0x2C, 0), ("i32.load8_u", 0x2D, 0), ("i32.load16_s", 0x2E, 1),
    ("i32.load16_u", 0x2F, 1), ("i64.load8_s", 0x30, 0), ("i64.load8_u", 0x31, 0),
    ("i64.load16_s", 0x32, 1), ("i64.load16_u", 0x33, 1), ("i64.load32_s", 0x34, 2),
    ("i64.load32_u", 0x35, 2), ("i32.store", 0x36, 2), ("i64.store", 0x37, 3),
    ("f32.store", 0x38, 2), ("f64.store", 0x39, 3), ("i32.store8", 0x3A, 0),
    ("i32.store16", 0x3B, 1), ("i64.store8", 0x3C, 0), ("i64.store16", 0x3D, 1),
    ("i64.store32", 0x3E, 2),
]:
    _op(_n, _c, MEM, _a)

_simple = """
45 i32.eqz 46 i32.eq 47 i32.ne 48 i32.lt_s 49 i32.lt_u 4A i32.gt_s 4B i32.gt_u 4C i32.le_s
4D i32.le_u 4E i32.ge_s 4F i32.ge_u 50 i64.eqz 51 i64.eq 52 i64.ne 53 i64.lt_s 54 i64.lt_u
55 i64.gt_s 56 i64.gt_u 57 i64.le_s 58 i64.le_u 59 i64.ge_s 5A i64.ge_u 5B f32.eq 5C f32.ne
5D f32.lt 5E f32.gt 5F f32.le 60 f32.ge 61 f64.eq 62 f64.ne 63 f64.lt 64 f64.gt 65 f64.le
66 f64.ge 67 i32.clz 68 i32.ctz 69 i32.popcnt 6A i32.add 6B i32.sub 6C i32.mul 6D i32.div_s
6E i32.div_u 6F i32.rem_s 70 i32.rem_u 71 i32.and 72 i32.or 73 i32.xor 74 i32.shl 75 i32.shr_s
76 i32.shr_u 77 i32.rotl 78 i32.rotr 79 i64.clz 7A i64.ctz 7B i64.popcnt 7C i64.add 7D i64.sub
7E i64.mul 7F i64.div_s 80 i64.div_u 81 i64.rem_s 82 i64.rem_u 83 i64.and 84 i64.or 85 i64.xor
86 i64.shl 87 i64.shr_s 88 i64.shr_u 89 i64.rotl 8A i64.rotr 8B f32.abs 8C f32.neg 8D f32.ceil
8E f32.floor 8F f32.trunc 90 f32.nearest 91 f32.sqrt 92 f32.add 93 f32.sub 94 f32.mul 95 f32.div
96 f32.min 97 f32.max 98 f32.copysign 99 f64.abs 9A f64.neg 9B f64.ceil 9C f64.floor 9D f64.trunc
9E f64.nearest 9F f64.sqrt A0 f64.add A1 f64.sub A2 f64.mul A3 f64.div A4 f64.min A5 f64.max
A6 f64.copysign A7 i32.wrap_i64 A8 i32.trunc_f32_s A9 i32.trunc_f32_u AA i32.trunc_f64_s
AB i32.trunc_f64_u AC i64.extend_i32_s AD i64.extend_i32_u AE i64.trunc_f32_s AF i64.trunc_f32_u
B0 i64.trunc_f64_s B1 i64.trunc_f64_u B2 f32.convert_i32_s B3 f32.convert_i32_u
B4 f32.convert_i64_s B5 f32.convert_i64_u B6 f32.demote_f64 B7 f64.convert_i32_s
B8 f64.convert_i32_u B9 f64.convert_i64_s BA f64.convert_i64_u BB f64.promote_f32
BC i32.reinterpret_f32 BD i64.reinterpret_f64 BE f32.reinterpret_i32 BF f64.reinterpret_i64
C0 i32.extend8_s C1 i32.extend16_s C2 i64.extend8_s C3 i64.extend16_s C4 i64.extend32_s
"""
_t = _simple.split()
for _i in range(0, len(_t), 2):
    _op(_t[_i + 1], int(_t[_i], 16))

# 0xFC prefix
for _n, _c, _i in [
    ("i32.trunc_sat_f32_s", 0, NONE), ("i32.trunc_sat_f32_u", 1, NONE),
    ("i32.trunc_sat_f64_s", 2, NONE), ("i32.trunc_sat_f64_u", 3, NONE),
    ("i64.trunc_sat_f32_s", 4, NONE), ("i64.trunc_sat_f32_u", 5, NONE),
    ("i64.trunc_sat_f64_s", 6, NONE), ("i64.trunc_sat_f64_u", 7, NONE),
    ("memory.init", 8, DATA), ("data.drop", 9, DATA | 0x100), ("memory.copy", 10, MEMMEM),
    ("memory.fill", 11, MEMIDX), ("table.init", 12, ELEM), ("elem.drop", 13, ELEM | 0x100),
    ("table.copy", 14, TWOIDX), ("table.grow", 15, TABLE), ("table.size", 16, TABLE),
    ("table.fill", 17, TABLE),
]:
    _op(_n, 0xFC00 | _c, _i)

# 0xFD prefix (SIMD128)
_simd_mem = [(0x00, "v128.load", 4), (0x01, "v128.load8x8_s", 3), (0x02, "v128.load8x8_u", 3),
             (0x03, "v128.load16x4_s", 3), (0x04, "v128.load16x4_u", 3),
             (0x05, "v128.load32x2_s", 3), (0x06, "v128.load32x2_u", 3),
             (0x07, "v128.load8_splat", 0), (0x08, "v128.load16_splat", 1),
             (0x09, "v128.load32_splat", 2), (0x0A, "v128.load64_splat", 3),
             (0x0B, "v128.store", 4), (0x5C, "v128.load32_zero", 2),
             (0x5D, "v128.load64_zero", 3)]
for _c, _n, _a in _simd_mem:
    _op(_n, 0xFD00 | _c, MEM, _a)
for _c, _n, _a in [(0x54, "v128.load8_lane", 0), (0x55, "v128.load16_lane", 1),
                   (0x56, "v128.load32_lane", 2), (0x57, "v128.load64_lane", 3),
                   (0x58, "v128.store8_lane", 0), (0x59, "v128.store16_lane", 1),
                   (0x5A, "v128.store32_lane", 2), (0x5B, "v128.store64_lane", 3)]:
    _op(_n, 0xFD00 | _c, MEMLANE, _a)
_op("v128.const", 0xFD0C, V128)
_op("i8x16.shuffle", 0xFD0D, SHUFFLE)
for _c, _n in [(0x15, "i8x16.extract_lane_s"), (0x16, "i8x16.extract_lane_u"),
               (0x17, "i8x16.replace_lane"), (0x18, "i16x8.extract_lane_s"),
               (0x19, "i16x8.extract_lane_u"), (0x1A, "i16x8.replace_lane"),
               (0x1B, "i32x4.extract_lane"), (0x1C, "i32x4.replace_lane"),
               (0x1D, "i64x2.extract_lane"), (0x1E, "i64x2.replace_lane"),
               (0x1F, "f32x4.extract_lane"), (0x20, "f32x4.replace_lane"),
               (0x21, "f64x2.extract_lane"), (0x22, "f64x2.replace_lane")]:
    _op(_n, 0xFD00 | _c, LANE)
_simd = """
0E i8x16.swizzle 0F i8x16.splat 10 i16x8.splat 11 i32x4.splat 12 i64x2.splat 13 f32x4.splat
14 f64x2.splat 23 i8x16.eq 24 i8x16.ne 25 i8x16.lt_s 26 i8x16.lt_u 27 i8x16.gt_s 28 i8x16.gt_u
29 i8x16.le_s 2A i8x16.le_u 2B i8x16.ge_s 2C i8x16.ge_u 2D i16x8.eq 2E i16x8.ne 2F i16x8.lt_s
30 i16x8.lt_u 31 i16x8.gt_s 32 i16x8.gt_u 33 i16x8.le_s 34 i16x8.le_u 35 i16x8.ge_s 36 i16x8.ge_u
37 i32x4.eq 38 i32x4.ne 39 i32x4.lt_s 3A i32x4.lt_u 3B i32x4.gt_s 3C i32x4.gt_u 3D i32x4.le_s
3E i32x4.le_u 3F i32x4.ge_s 40 i32x4.ge_u 41 f32x4.eq 42 f32x4.ne 43 f32x4.lt 44 f32x4.gt
45 f32x4.le 46 f32x4.ge 47 f64x2.eq 48 f64x2.ne 49 f64x2.lt 4A f64x2.gt 4B f64x2.le 4C f64x2.ge
4D v128.not 4E v128.and 4F v128.andnot 50 v128.or 51 v128.xor 52 v128.bitselect 53 v128.any_true
5E f32x4.demote_f64x2_zero 5F f64x2.promote_low_f32x4
60 i8x16.abs 61 i8x16.neg 62 i8x16.popcnt 63 i8x16.all_true 64 i8x16.bitmask
65 i8x16.narrow_i16x8_s 66 i8x16.narrow_i16x8_u 67 f32x4.ceil 68 f32x4.floor 69 f32x4.trunc
6A f32x4.nearest 6B i8x16.shl 6C i8x16.shr_s 6D i8x16.shr_u 6E i8x16.add 6F i8x16.add_sat_s
70 i8x16.add_sat_u 71 i8x16.sub 72 i8x16.sub_sat_s 73 i8x16.sub_sat_u 74 f64x2.ceil 75 f64x2.floor
76 i8x16.min_s 77 i8x16.min_u 78 i8x16.max_s 79 i8x16.max_u 7A f64x2.trunc 7B i8x16.avgr_u
7C i16x8.extadd_pairwise_i8x16_s 7D i16x8.extadd_pairwise_i8x16_u
7E i32x4.extadd_pairwise_i16x8_s 7F i32x4.extadd_pairwise_i16x8_u
80 i16x8.abs 81 i16x8.neg 82 i16x8.q15mulr_sat_s 83 i16x8.all_true 84 i16x8.bitmask
85 i16x8.narrow_i32x4_s 86 i16x8.narrow_i32x4_u 87 i16x8.extend_low_i8x16_s
88 i16x8.extend_high_i8x16_s 89 i16x8.extend_low_i8x16_u 8A i16x8.extend_high_i8x16_u
8B i16x8.shl 8C i16x8.shr_s 8D i16x8.shr_u 8E i16x8.add 8F i16x8.add_sat_s 90 i16x8.add_sat_u
91 i16x8.sub 92 i16x8.sub_sat_s 93 i16x8.sub_sat_u 94 f64x2.nearest 95 i16x8.mul 96 i16x8.min_s
97 i16x8.min_u 98 i16x8.max_s 99 i16x8.max_u 9B i16x8.avgr_u 9C i16x8.extmul_low_i8x16_s
9D i16x8.extmul_high_i8x16_s 9E i16x8.extmul_low_i8x16_u 9F i16x8.extmul_high_i8x16_u
A0 i32x4.abs A1 i32x4.neg A3 i32x4.all_true A4 i32x4.bitmask A7 i32x4.extend_low_i16x8_s
A8 i32x4.extend_high_i16x8_s A9 i32x4.extend_low_i16x8_u AA i32x4.extend_high_i16x8_u
AB i32x4.shl AC i32x4.shr_s AD i32x4.shr_u AE i32x4.add B1 i32x4.sub B5 i32x4.mul B6 i32x4.min_s
B7 i32x4.min_u B8 i32x4.max_s B9 i32x4.max_u BA i32x4.dot_i16x8_s BC i32x4.extmul_low_i16x8_s
BD i32x4.extmul_high_i16x8_s BE i32x4.extmul_low_i16x8_u BF i32x4.extmul_high_i16x8_u
C0 i64x2.abs C1 i64x2.neg C3 i64x2.all_true C4 i64x2.bitmask C7 i64x2.extend_low_i32x4_s
C8 i64x2.extend_high_i32x4_s C9 i64x2.extend_low_i32x4_u CA i64x2.extend_high_i32x4_u
CB i64x2.shl CC i64x2.shr_s CD i64x2.shr_u CE i64x2.add D1 i64x2.sub D5 i64x2.mul D6 i64x2.eq
D7 i64x2.ne D8 i64x2.lt_s D9 i64x2.gt_s DA i64x2.le_s DB i64x2.ge_s DC i64x2.extmul_low_i32x4_s
DD i64x2.extmul_high_i32x4_s DE i64x2.extmul_low_i32x4_u DF i64x2.extmul_high_i32x4_u
E0 f32x4.abs E1 f32x4.neg E3 f32x4.sqrt E4 f32x4.add E5 f32x4.sub E6 f32x4.mul E7 f32x4.div
E8 f32x4.min E9 f32x4.max EA f32x4.pmin EB f32x4.pmax EC f64x2.abs ED f64x2.neg EF f64x2.sqrt
F0 f64x2.add F1 f64x2.sub F2 f64x2.mul F3 f64x2.div F4 f64x2.min F5 f64x2.max F6 f64x2.pmin
F7 f64x2.pmax F8 i32x4.trunc_sat_f32x4_s F9 i32x4.trunc_sat_f32x4_u FA f32x4.convert_i32x4_s
FB f32x4.convert_i32x4_u FC i32x4.trunc_sat_f64x2_s_zero FD i32x4.trunc_sat_f64x2_u_zero
FE f64x2.convert_low_i32x4_s FF f64x2.convert_low_i32x4_u
"""
_t = _simd.split()
for _i in range(0, len(_t), 2):
    _op(_t[_i + 1], 0xFD00 | int(_t[_i], 16))

# legacy aliases used by older .wat files (e.g. the reference's fibonacci.wat)
ALIASES = {"get_local": "local.get", "set_local": "local.set", "tee_local": "local.tee",
           "get_global": "global.get", "set_global": "global.set"}

VALTYPES = {"i32": 0x7F, "i64": 0x7E, "f32": 0x7D, "f64": 0x7C, "v128": 0x7B,
            "funcref": 0x70, "externref": 0x6F, "anyfunc": 0x70}
