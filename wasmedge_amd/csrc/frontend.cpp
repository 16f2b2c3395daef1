// frontend.cpp -- decode + validate + lower a wasm module to the register-form DBC.
// See frontend.h / dbc.h. Reference behaviour restated (with file:line) where it
// determines results or instruction counts.
#include "frontend.h"

#include <cstring>
#include <map>
#include <unordered_map>

namespace wb {

namespace {

// ErrCodes (include/common/enum.inc:573-749)
enum : uint8_t { E_MALFORMED = 0x21, E_ILLEGAL_OPCODE = 0x37, E_TYPECHECK = 0x41,
                 E_UNSUPPORTED = 0x02 /* RuntimeError: outside the batched subset */ };

struct Err {
  uint8_t code;
  std::string msg;
};
struct NeedMutTables {};

struct Reader {
  const uint8_t *p, *end;
  uint8_t u8() {
    if (p >= end) throw Err{E_MALFORMED, "unexpected end"};
    return *p++;
  }
  uint64_t uleb(int bits = 32) {
    uint64_t v = 0;
    int sh = 0;
    for (;;) {
      uint8_t b = u8();
      v |= uint64_t(b & 0x7F) << sh;
      sh += 7;
      if (!(b & 0x80)) break;
      if (sh >= bits + 7) throw Err{E_MALFORMED, "integer representation too long"};
    }
    return v;
  }
  int64_t sleb(int bits) {
    uint64_t v = 0;   // unsigned accumulation: shifting into bit 63 is defined
    int sh = 0;
    uint8_t b;
    do {
      b = u8();
      if (sh < 64) v |= uint64_t(b & 0x7F) << sh;
      sh += 7;
      if (sh >= bits + 7) throw Err{E_MALFORMED, "integer representation too long"};
    } while (b & 0x80);
    if (sh < 64 && (b & 0x40)) v |= ~uint64_t(0) << sh;
    return int64_t(v);
  }
  uint32_t u32() { return uint32_t(uleb(32)); }
  std::string name() {
    uint32_t n = u32();
    if (uint64_t(end - p) < n) throw Err{E_MALFORMED, "name"};
    std::string s(reinterpret_cast<const char *>(p), n);
    p += n;
    return s;
  }
};

// ------------------------------------------------------------------ op tables
struct SimpleOp {
  uint16_t dop;
  int16_t dop_imm;     // register-immediate variant, -1 if none
  const char *sig;     // "pops:pushes", i=i32 l=i64 f=f32 d=f64 v=v128
  bool commutative;
  uint32_t imm = 0;    // OP_V_BINX / OP_V_UNX: the 0xFD sub-opcode
};

std::unordered_map<uint16_t, SimpleOp> build_simple() {
  std::unordered_map<uint16_t, SimpleOp> t;
  auto add = [&](uint16_t w, uint16_t d, int16_t di, const char *s, bool c = false) {
    t[w] = SimpleOp{d, di, s, c};
  };
  // i32 compare / arithmetic (wasm 0x46-0x4F, 0x6A-0x78)
  const uint16_t i32cmp[] = {OP_I32_EQ, OP_I32_NE, OP_I32_LT_S, OP_I32_LT_U, OP_I32_GT_S,
                             OP_I32_GT_U, OP_I32_LE_S, OP_I32_LE_U, OP_I32_GE_S, OP_I32_GE_U};
  for (int k = 0; k < 10; k++)
    add(0x46 + k, i32cmp[k], int16_t(i32cmp[k] - OP_I32_ADD + OP_I32_ADD_I), "ii:i", k < 2);
  const uint16_t i32ar[] = {OP_I32_ADD, OP_I32_SUB, OP_I32_MUL, OP_I32_DIV_S, OP_I32_DIV_U,
                            OP_I32_REM_S, OP_I32_REM_U, OP_I32_AND, OP_I32_OR, OP_I32_XOR,
                            OP_I32_SHL, OP_I32_SHR_S, OP_I32_SHR_U, OP_I32_ROTL, OP_I32_ROTR};
  const bool i32c[] = {1, 0, 1, 0, 0, 0, 0, 1, 1, 1, 0, 0, 0, 0, 0};
  for (int k = 0; k < 15; k++)
    add(0x6A + k, i32ar[k], int16_t(i32ar[k] - OP_I32_ADD + OP_I32_ADD_I), "ii:i", i32c[k]);
  const uint16_t i64cmp[] = {OP_I64_EQ, OP_I64_NE, OP_I64_LT_S, OP_I64_LT_U, OP_I64_GT_S,
                             OP_I64_GT_U, OP_I64_LE_S, OP_I64_LE_U, OP_I64_GE_S, OP_I64_GE_U};
  for (int k = 0; k < 10; k++)
    add(0x51 + k, i64cmp[k], int16_t(i64cmp[k] - OP_I64_ADD + OP_I64_ADD_I), "ll:i", k < 2);
  const uint16_t i64ar[] = {OP_I64_ADD, OP_I64_SUB, OP_I64_MUL, OP_I64_DIV_S, OP_I64_DIV_U,
                            OP_I64_REM_S, OP_I64_REM_U, OP_I64_AND, OP_I64_OR, OP_I64_XOR,
                            OP_I64_SHL, OP_I64_SHR_S, OP_I64_SHR_U, OP_I64_ROTL, OP_I64_ROTR};
  for (int k = 0; k < 15; k++)
    add(0x7C + k, i64ar[k], int16_t(i64ar[k] - OP_I64_ADD + OP_I64_ADD_I), "ll:l", i32c[k]);
  add(0x45, OP_I32_EQZ, -1, "i:i");
  add(0x50, OP_I64_EQZ, -1, "l:i");
  add(0x67, OP_I32_CLZ, -1, "i:i"); add(0x68, OP_I32_CTZ, -1, "i:i");
  add(0x69, OP_I32_POPCNT, -1, "i:i");
  add(0x79, OP_I64_CLZ, -1, "l:l"); add(0x7A, OP_I64_CTZ, -1, "l:l");
  add(0x7B, OP_I64_POPCNT, -1, "l:l");
  const uint16_t f32cmp[] = {OP_F32_EQ, OP_F32_NE, OP_F32_LT, OP_F32_GT, OP_F32_LE, OP_F32_GE};
  const uint16_t f64cmp[] = {OP_F64_EQ, OP_F64_NE, OP_F64_LT, OP_F64_GT, OP_F64_LE, OP_F64_GE};
  for (int k = 0; k < 6; k++) { add(0x5B + k, f32cmp[k], -1, "ff:i"); add(0x61 + k, f64cmp[k], -1, "dd:i"); }
  const uint16_t f32un[] = {OP_F32_ABS, OP_F32_NEG, OP_F32_CEIL, OP_F32_FLOOR, OP_F32_TRUNC,
                            OP_F32_NEAREST, OP_F32_SQRT};
  const uint16_t f64un[] = {OP_F64_ABS, OP_F64_NEG, OP_F64_CEIL, OP_F64_FLOOR, OP_F64_TRUNC,
                            OP_F64_NEAREST, OP_F64_SQRT};
  for (int k = 0; k < 7; k++) { add(0x8B + k, f32un[k], -1, "f:f"); add(0x99 + k, f64un[k], -1, "d:d"); }
  const uint16_t f32bin[] = {OP_F32_ADD, OP_F32_SUB, OP_F32_MUL, OP_F32_DIV, OP_F32_MIN,
                             OP_F32_MAX, OP_F32_COPYSIGN};
  const uint16_t f64bin[] = {OP_F64_ADD, OP_F64_SUB, OP_F64_MUL, OP_F64_DIV, OP_F64_MIN,
                             OP_F64_MAX, OP_F64_COPYSIGN};
  for (int k = 0; k < 7; k++) { add(0x92 + k, f32bin[k], -1, "ff:f"); add(0xA0 + k, f64bin[k], -1, "dd:d"); }
  add(0xA8, OP_I32_TRUNC_F32_S, -1, "f:i"); add(0xA9, OP_I32_TRUNC_F32_U, -1, "f:i");
  add(0xAA, OP_I32_TRUNC_F64_S, -1, "d:i"); add(0xAB, OP_I32_TRUNC_F64_U, -1, "d:i");
  add(0xAC, OP_I64_EXTEND_I32_S, -1, "i:l"); add(0xAD, OP_I64_EXTEND_I32_U, -1, "i:l");
  add(0xAE, OP_I64_TRUNC_F32_S, -1, "f:l"); add(0xAF, OP_I64_TRUNC_F32_U, -1, "f:l");
  add(0xB0, OP_I64_TRUNC_F64_S, -1, "d:l"); add(0xB1, OP_I64_TRUNC_F64_U, -1, "d:l");
  add(0xB2, OP_F32_CONVERT_I32_S, -1, "i:f"); add(0xB3, OP_F32_CONVERT_I32_U, -1, "i:f");
  add(0xB4, OP_F32_CONVERT_I64_S, -1, "l:f"); add(0xB5, OP_F32_CONVERT_I64_U, -1, "l:f");
  add(0xB6, OP_F32_DEMOTE_F64, -1, "d:f");
  add(0xB7, OP_F64_CONVERT_I32_S, -1, "i:d"); add(0xB8, OP_F64_CONVERT_I32_U, -1, "i:d");
  add(0xB9, OP_F64_CONVERT_I64_S, -1, "l:d"); add(0xBA, OP_F64_CONVERT_I64_U, -1, "l:d");
  add(0xBB, OP_F64_PROMOTE_F32, -1, "f:d");
  add(0xC0, OP_I32_EXT8S, -1, "i:i"); add(0xC1, OP_I32_EXT16S, -1, "i:i");
  add(0xC2, OP_I64_EXT8S, -1, "l:l"); add(0xC3, OP_I64_EXT16S, -1, "l:l");
  add(0xC4, OP_I64_EXT32S, -1, "l:l");
  const uint16_t sat[] = {OP_I32_TRUNC_SAT_F32_S, OP_I32_TRUNC_SAT_F32_U, OP_I32_TRUNC_SAT_F64_S,
                          OP_I32_TRUNC_SAT_F64_U, OP_I64_TRUNC_SAT_F32_S, OP_I64_TRUNC_SAT_F32_U,
                          OP_I64_TRUNC_SAT_F64_S, OP_I64_TRUNC_SAT_F64_U};
  const char *satsig[] = {"f:i", "f:i", "d:i", "d:i", "f:l", "f:l", "d:l", "d:l"};
  for (int k = 0; k < 8; k++) add(0xFC00 + k, sat[k], -1, satsig[k]);
  // SIMD128 (engine.cpp:748-1609): ops with a dedicated DOp
  add(0xFD4D, OP_V_NOT, -1, "v:v"); add(0xFD4E, OP_V_AND, -1, "vv:v", true);
  add(0xFD4F, OP_V_ANDNOT, -1, "vv:v"); add(0xFD50, OP_V_OR, -1, "vv:v", true);
  add(0xFD51, OP_V_XOR, -1, "vv:v", true); add(0xFD52, OP_V_BITSELECT, -1, "vvv:v");
  add(0xFD53, OP_V_ANY_TRUE, -1, "v:i");
  add(0xFD0F, OP_V_I8X16_SPLAT, -1, "i:v"); add(0xFD10, OP_V_I16X8_SPLAT, -1, "i:v");
  add(0xFD11, OP_V_I32X4_SPLAT, -1, "i:v"); add(0xFD12, OP_V_I64X2_SPLAT, -1, "l:v");
  add(0xFD13, OP_V_F32X4_SPLAT, -1, "f:v"); add(0xFD14, OP_V_F64X2_SPLAT, -1, "d:v");
  add(0xFD0E, OP_V_SWIZZLE, -1, "vv:v");
  add(0xFD6E, OP_V_I8X16_ADD, -1, "vv:v"); add(0xFD71, OP_V_I8X16_SUB, -1, "vv:v");
  add(0xFD8E, OP_V_I16X8_ADD, -1, "vv:v"); add(0xFD91, OP_V_I16X8_SUB, -1, "vv:v");
  add(0xFD95, OP_V_I16X8_MUL, -1, "vv:v");
  add(0xFDAE, OP_V_I32X4_ADD, -1, "vv:v"); add(0xFDB1, OP_V_I32X4_SUB, -1, "vv:v");
  add(0xFDB5, OP_V_I32X4_MUL, -1, "vv:v");
  add(0xFDCE, OP_V_I64X2_ADD, -1, "vv:v"); add(0xFDD1, OP_V_I64X2_SUB, -1, "vv:v");
  add(0xFDD5, OP_V_I64X2_MUL, -1, "vv:v");
  add(0xFD23, OP_V_I8X16_EQ, -1, "vv:v"); add(0xFD24, OP_V_I8X16_NE, -1, "vv:v");
  add(0xFD2D, OP_V_I16X8_EQ, -1, "vv:v"); add(0xFD2E, OP_V_I16X8_NE, -1, "vv:v");
  const uint16_t i32x4cmp[] = {OP_V_I32X4_EQ, OP_V_I32X4_NE, OP_V_I32X4_LT_S, OP_V_I32X4_LT_U,
                               OP_V_I32X4_GT_S, OP_V_I32X4_GT_U, OP_V_I32X4_LE_S,
                               OP_V_I32X4_LE_U, OP_V_I32X4_GE_S, OP_V_I32X4_GE_U};
  for (int k = 0; k < 10; k++) add(0xFD37 + k, i32x4cmp[k], -1, "vv:v");
  const uint16_t i64x2cmp[] = {OP_V_I64X2_EQ, OP_V_I64X2_NE, OP_V_I64X2_LT_S, OP_V_I64X2_GT_S,
                               OP_V_I64X2_LE_S, OP_V_I64X2_GE_S};
  for (int k = 0; k < 6; k++) add(0xFDD6 + k, i64x2cmp[k], -1, "vv:v");
  const uint16_t shifts[] = {OP_V_I8X16_SHL, OP_V_I8X16_SHR_S, OP_V_I8X16_SHR_U};
  for (int k = 0; k < 3; k++) add(0xFD6B + k, shifts[k], -1, "vi:v");
  add(0xFD8B, OP_V_I16X8_SHL, -1, "vi:v"); add(0xFD8C, OP_V_I16X8_SHR_S, -1, "vi:v");
  add(0xFD8D, OP_V_I16X8_SHR_U, -1, "vi:v");
  add(0xFDAB, OP_V_I32X4_SHL, -1, "vi:v"); add(0xFDAC, OP_V_I32X4_SHR_S, -1, "vi:v");
  add(0xFDAD, OP_V_I32X4_SHR_U, -1, "vi:v");
  add(0xFDCB, OP_V_I64X2_SHL, -1, "vi:v"); add(0xFDCC, OP_V_I64X2_SHR_S, -1, "vi:v");
  add(0xFDCD, OP_V_I64X2_SHR_U, -1, "vi:v");
  add(0xFD63, OP_V_I8X16_ALL_TRUE, -1, "v:i"); add(0xFD83, OP_V_I16X8_ALL_TRUE, -1, "v:i");
  add(0xFDA3, OP_V_I32X4_ALL_TRUE, -1, "v:i"); add(0xFDC3, OP_V_I64X2_ALL_TRUE, -1, "v:i");
  add(0xFD64, OP_V_I8X16_BITMASK, -1, "v:i"); add(0xFD84, OP_V_I16X8_BITMASK, -1, "v:i");
  add(0xFDA4, OP_V_I32X4_BITMASK, -1, "v:i"); add(0xFDC4, OP_V_I64X2_BITMASK, -1, "v:i");
  add(0xFDA1, OP_V_I32X4_NEG, -1, "v:v"); add(0xFDC1, OP_V_I64X2_NEG, -1, "v:v");
  add(0xFDA0, OP_V_I32X4_ABS, -1, "v:v"); add(0xFDC0, OP_V_I64X2_ABS, -1, "v:v");
  const uint16_t f32x4b[] = {OP_V_F32X4_ADD, OP_V_F32X4_SUB, OP_V_F32X4_MUL, OP_V_F32X4_DIV,
                             OP_V_F32X4_MIN, OP_V_F32X4_MAX, OP_V_F32X4_PMIN, OP_V_F32X4_PMAX};
  const uint16_t f64x2b[] = {OP_V_F64X2_ADD, OP_V_F64X2_SUB, OP_V_F64X2_MUL, OP_V_F64X2_DIV,
                             OP_V_F64X2_MIN, OP_V_F64X2_MAX, OP_V_F64X2_PMIN, OP_V_F64X2_PMAX};
  for (int k = 0; k < 8; k++) { add(0xFDE4 + k, f32x4b[k], -1, "vv:v"); add(0xFDF0 + k, f64x2b[k], -1, "vv:v"); }
  const uint16_t f32x4c[] = {OP_V_F32X4_EQ, OP_V_F32X4_NE, OP_V_F32X4_LT, OP_V_F32X4_GT,
                             OP_V_F32X4_LE, OP_V_F32X4_GE};
  const uint16_t f64x2c[] = {OP_V_F64X2_EQ, OP_V_F64X2_NE, OP_V_F64X2_LT, OP_V_F64X2_GT,
                             OP_V_F64X2_LE, OP_V_F64X2_GE};
  for (int k = 0; k < 6; k++) { add(0xFD41 + k, f32x4c[k], -1, "vv:v"); add(0xFD47 + k, f64x2c[k], -1, "vv:v"); }
  add(0xFDE0, OP_V_F32X4_ABS, -1, "v:v"); add(0xFDE1, OP_V_F32X4_NEG, -1, "v:v");
  add(0xFDE3, OP_V_F32X4_SQRT, -1, "v:v");
  add(0xFDEC, OP_V_F64X2_ABS, -1, "v:v"); add(0xFDED, OP_V_F64X2_NEG, -1, "v:v");
  add(0xFDEF, OP_V_F64X2_SQRT, -1, "v:v");
  // the remaining lane-wise SIMD ops share two generic DOps keyed by the sub-opcode
  // (binary_numeric.ipp:203-567, unary_numeric.ipp:98-415, engine.cpp:748-1609)
  auto addx = [&](uint16_t w, uint16_t d, const char *s) { t[w] = SimpleOp{d, -1, s, false, uint32_t(w & 0xFF)}; };
  const uint8_t binx[] = {0x25, 0x26, 0x27, 0x28, 0x29, 0x2A, 0x2B, 0x2C,   // i8x16 lt..ge
                          0x2F, 0x30, 0x31, 0x32, 0x33, 0x34, 0x35, 0x36,   // i16x8 lt..ge
                          0x65, 0x66, 0x85, 0x86,                           // narrow
                          0x6F, 0x70, 0x72, 0x73, 0x76, 0x77, 0x78, 0x79, 0x7B,
                          0x82, 0x8F, 0x90, 0x92, 0x93, 0x96, 0x97, 0x98, 0x99, 0x9B,
                          0x9C, 0x9D, 0x9E, 0x9F,                           // i16x8 extmul
                          0xB6, 0xB7, 0xB8, 0xB9, 0xBA, 0xBC, 0xBD, 0xBE, 0xBF,
                          0xDC, 0xDD, 0xDE, 0xDF};                          // i64x2 extmul
  for (uint8_t w : binx) addx(0xFD00 | w, OP_V_BINX, "vv:v");
  const uint8_t unx[] = {0x5E, 0x5F, 0x60, 0x61, 0x62, 0x67, 0x68, 0x69, 0x6A, 0x74, 0x75,
                         0x7A, 0x94, 0x7C, 0x7D, 0x7E, 0x7F, 0x80, 0x81, 0x87, 0x88, 0x89,
                         0x8A, 0xA7, 0xA8, 0xA9, 0xAA, 0xC7, 0xC8, 0xC9, 0xCA, 0xF8, 0xF9,
                         0xFA, 0xFB, 0xFC, 0xFD, 0xFE, 0xFF};
  for (uint8_t w : unx) addx(0xFD00 | w, OP_V_UNX, "v:v");
  return t;
}

const std::unordered_map<uint16_t, SimpleOp> &simple_ops() {
  static const auto t = build_simple();
  return t;
}

uint8_t sigt(char c) {
  switch (c) {
    case 'i': return I32; case 'l': return I64; case 'f': return F32; case 'd': return F64;
    default: return V128;
  }
}

bool is_numtype(uint8_t t) {
  return t == I32 || t == I64 || t == F32 || t == F64 || t == V128 || t == FUNCREF ||
         t == EXTERNREF;
}

// ------------------------------------------------------------------ lowering
enum Kind : uint8_t { K_CELL, K_CONST, K_LOCAL };

struct Entry {
  uint8_t type;
  Kind kind;
  uint32_t cell;        // canonical cell of this stack slot
  uint32_t local;       // K_LOCAL: local index
  uint32_t k[4];        // K_CONST: value words
  int64_t producer;     // index of the DInstr that wrote this cell as `c`, -1 if none
  bool var = true;      // may differ between instances (Program::divergent_mem analysis)
};

struct Fixup {
  bool brtab;           // patch brtab entry (else DInstr imm/d)
  uint32_t index;
  int32_t extra;
};

enum CtrlKind : uint8_t { C_BLOCK, C_LOOP, C_IF, C_FUNC };

struct Ctrl {
  CtrlKind kind;
  std::vector<uint8_t> in, out;
  uint32_t height;       // stack entries below the frame's values
  uint32_t cell_base;    // canonical cell at height
  bool unreachable = false;
  bool dead = false;     // pushed inside unreachable code
  bool label_known = false;
  uint32_t label_pc = 0;
  int32_t label_tcnt = 0;
  std::vector<Fixup> fixups;
  int64_t else_br = -1;  // BR_UNLESS of an `if`, patched at else/end
  bool has_else = false;
};

struct CallFix {
  uint32_t instr;
  uint32_t callee;
};

// Which locals may hold per-instance values, by function (flow-insensitive): the
// parameters of functions the host or call_indirect can call, every local ever set from
// a parameter / loaded value / mutable global / call result, and (interprocedurally) the
// parameters some call site passes such a value. Lowering repeats until it is stable;
// Program::divergent_mem then says whether a load/store address can depend on one.
struct VarInfo {
  std::vector<std::vector<uint8_t>> locals;
  bool changed = false;
};

class Lowerer {
 public:
  Lowerer(Program &P, const uint8_t *bin, VarInfo &vi) : P(P), bin(bin), vi(vi) {}

  void lower_function(uint32_t fi, std::vector<CallFix> &callfix);

 private:
  Program &P;
  const uint8_t *bin;
  VarInfo &vi;
  uint32_t cur_fn = 0;
  void set_var_local(uint32_t f, uint32_t li) {
    if (!vi.locals[f][li]) { vi.locals[f][li] = 1; vi.changed = true; }
  }
  // per function
  const FuncType *ft = nullptr;
  std::vector<uint8_t> ltypes;
  std::vector<uint32_t> lcell;
  uint32_t frame_base = 0, opnd_base = 0, max_cell = 0;
  std::vector<Entry> st;
  std::vector<Ctrl> ctrl;
  uint32_t pending = 0;
  std::vector<uint16_t> pend_ops;   // the opcodes behind `pending`, in order (Program::dops)
  int64_t last_emit = -1;
  bool can_retarget = false;
  std::vector<CallFix> *callfix = nullptr;

  [[noreturn]] void fail(uint8_t code, const std::string &m) { throw Err{code, m}; }
  // a table-mutating op in a module lowered for a shared immutable table: start over
  // with per-lane tables (parse_and_lower catches this)
  void need_mut_tables() { if (!P.mut_tables) throw NeedMutTables{}; }

  bool live() const { return !ctrl.back().unreachable; }

  uint32_t top_cell() const {
    if (st.empty()) return opnd_base;
    return st.back().cell + cells_of(st.back().type);
  }

  static bool is_ctl(uint16_t op) {
    switch (op) {
      case OP_JMP: case OP_BR_IF: case OP_BR_UNLESS: case OP_BR_IF_MOV1: case OP_BR_IF_MOV2:
      case OP_BR_TABLE: case OP_CALL: case OP_CALL_INDIRECT: case OP_RET: case OP_UNREACHABLE:
      case OP_HOST_CALL: case OP_TAIL_CALL: case OP_TAIL_CALL_INDIRECT:
      case OP_I32_DIV_S: case OP_I32_DIV_U: case OP_I32_REM_S: case OP_I32_REM_U:
      case OP_I32_DIV_S_I: case OP_I32_DIV_U_I: case OP_I32_REM_S_I: case OP_I32_REM_U_I:
      case OP_I64_DIV_S: case OP_I64_DIV_U: case OP_I64_REM_S: case OP_I64_REM_U:
      case OP_I64_DIV_S_I: case OP_I64_DIV_U_I: case OP_I64_REM_S_I: case OP_I64_REM_U_I:
      case OP_I32_TRUNC_F32_S: case OP_I32_TRUNC_F32_U: case OP_I32_TRUNC_F64_S:
      case OP_I32_TRUNC_F64_U: case OP_I64_TRUNC_F32_S: case OP_I64_TRUNC_F32_U:
      case OP_I64_TRUNC_F64_S: case OP_I64_TRUNC_F64_U:
      case OP_LD8S32: case OP_LD8U32: case OP_LD16S32: case OP_LD16U32: case OP_LD32:
      case OP_LD8S64: case OP_LD8U64: case OP_LD16S64: case OP_LD16U64: case OP_LD32S64:
      case OP_LD32U64: case OP_LD64: case OP_LD128: case OP_ST8: case OP_ST16: case OP_ST32:
      case OP_ST64: case OP_ST128: case OP_MEM_FILL: case OP_MEM_COPY: case OP_MEM_INIT:
      case OP_TABLE_GET: case OP_TABLE_SET: case OP_TABLE_SIZE: case OP_TABLE_GROW:
      case OP_TABLE_FILL: case OP_TABLE_COPY: case OP_TABLE_INIT: case OP_ELEM_DROP:
      case OP_V_LD8X8S: case OP_V_LD8X8U: case OP_V_LD16X4S:
      case OP_V_LD16X4U: case OP_V_LD32X2S: case OP_V_LD32X2U: case OP_V_LD8SPLAT:
      case OP_V_LD16SPLAT: case OP_V_LD32SPLAT: case OP_V_LD64SPLAT: case OP_V_LD32ZERO:
      case OP_V_LD64ZERO: case OP_V_LDLANE: case OP_V_STLANE:
      case OP_XLD: case OP_XST: case OP_XLANE: case OP_XMEM_FILL: case OP_XMEM_COPY: case OP_XMEM_INIT:
        return true;
      default:
        return op >= OP_BR_EQ && op <= OP_BR_GE_U_I;
    }
  }

  DInstr &emit(uint16_t op, uint32_t a = 0, uint32_t b = 0, uint32_t c = 0, uint32_t d = 0,
               uint32_t imm = 0) {
    if (a > 0xFFFF || b > 0xFFFF || c > 0xFFFF)
      fail(E_UNSUPPORTED, "cell index out of range for the DBC encoding");
    spill_pending();                         // cnt is 8 bits
    DInstr I;
    I.w0 = uint32_t(op) | (pending << 16) | (is_ctl(op) ? DBC_CTL : 0u);
    I.w1 = (a & 0xFFFF) | (b << 16);
    I.w2 = (c & 0xFFFF) | (d << 16);
    I.w3 = imm;
    if (pending > P.max_wasm_instrs_per_dispatch) P.max_wasm_instrs_per_dispatch = pending;
    pending = 0;
    P.code.push_back(I);
    P.dops.push_back(std::move(pend_ops));
    pend_ops.clear();
    last_emit = int64_t(P.code.size()) - 1;
    can_retarget = true;
    return P.code.back();
  }

  // pending counts above 255 go into NOP_CNT carriers (255 each). Before a label too: a
  // branch to it skips the carriers (or, to a loop, does not re-run them), so its count
  // correction stays within [-255, 0] however many folded instructions precede the label
  // (40,000 nops before a loop once gave a correction that did not fit the 16-bit field).
  void spill_pending() {
    while (pending > 255) {
      P.code.push_back(DInstr{uint32_t(OP_NOP_CNT) | (255u << 16), 0, 0, 0});
      P.dops.emplace_back(pend_ops.begin(), pend_ops.begin() + 255);
      pend_ops.erase(pend_ops.begin(), pend_ops.begin() + 255);
      pending -= 255;
    }
  }
  void place_label() {
    can_retarget = false;
    spill_pending();
  }

  // ---------------- stack
  Entry &push_cell(uint8_t t, int64_t producer = -1) {
    Entry e{};
    e.type = t;
    e.kind = K_CELL;
    e.cell = top_cell();
    e.producer = producer;
    st.push_back(e);
    uint32_t hi = e.cell + cells_of(t);
    if (hi > max_cell) max_cell = hi;
    return st.back();
  }
  void push_const(uint8_t t, const uint32_t *k) {
    Entry &e = push_cell(t);
    e.kind = K_CONST;
    e.var = false;
    memcpy(e.k, k, sizeof e.k);
  }
  void push_local(uint32_t li) {
    Entry &e = push_cell(ltypes[li]);
    e.kind = K_LOCAL;
    e.local = li;
    e.var = vi.locals[cur_fn][li] != 0;
  }
  Entry pop_any() {
    Ctrl &f = ctrl.back();
    if (st.size() == f.height) {
      if (f.unreachable) {
        Entry e{};
        e.type = UNKNOWN;
        e.kind = K_CELL;
        e.cell = top_cell();
        e.producer = -1;
        return e;
      }
      fail(E_TYPECHECK, "type mismatch: operand stack underflow");
    }
    Entry e = st.back();
    st.pop_back();
    return e;
  }
  Entry pop_t(uint8_t t) {
    Entry e = pop_any();
    if (e.type != UNKNOWN && t != UNKNOWN && e.type != t) fail(E_TYPECHECK, "type mismatch");
    if (e.type == UNKNOWN) e.type = t;
    return e;
  }
  void pop_types(const std::vector<uint8_t> &ts) {
    for (size_t k = ts.size(); k > 0; k--) pop_t(ts[k - 1]);
  }

  // ---------------- materialisation
  void materialize_into(const Entry &e, uint32_t dst) {
    uint32_t w = cells_of(e.type);
    if (e.kind == K_CONST) {
      if (w == 1) emit(OP_CONST32, 0, 0, dst, 0, e.k[0]);
      else if (w == 2) emit(OP_CONST64, e.k[1] & 0xFFFF, e.k[1] >> 16, dst, 0, e.k[0]);
      else {
        uint32_t idx = uint32_t(P.vconst.size() / 4);
        P.vconst.insert(P.vconst.end(), e.k, e.k + 4);
        emit(OP_CONST128, 0, 0, dst, 0, idx);
      }
    } else {
      uint32_t src = e.kind == K_LOCAL ? lcell[e.local] : e.cell;
      if (src == dst) return;
      emit(w == 1 ? OP_MOV32 : w == 2 ? OP_MOV64 : OP_MOV128, src, 0, dst);
    }
  }
  void materialize(size_t idx) {
    Entry &e = st[idx];
    if (e.kind == K_CELL) return;
    if (live()) materialize_into(e, e.cell);
    e.kind = K_CELL;
    e.producer = -1;
  }
  void materialize_locals(int64_t local = -1) {
    for (size_t k = 0; k < st.size(); k++)
      if (st[k].kind == K_LOCAL && (local < 0 || st[k].local == uint32_t(local))) materialize(k);
  }
  void materialize_top(size_t n) {
    for (size_t k = st.size() - n; k < st.size(); k++) materialize(k);
  }
  // source cell for an operand (materialising constants into their own slot)
  uint32_t src(Entry &e) {
    if (e.kind == K_LOCAL) return lcell[e.local];
    if (e.kind == K_CONST) {
      if (live()) materialize_into(e, e.cell);
      e.kind = K_CELL;
    }
    return e.cell;
  }

  // ---------------- control
  void block_type(Reader &r, std::vector<uint8_t> &in, std::vector<uint8_t> &out) {
    uint8_t b = *r.p;
    if (b == 0x40) { r.p++; return; }
    if (is_numtype(b)) { r.p++; out.push_back(b); return; }
    int64_t ti = r.sleb(33);
    if (ti < 0 || uint64_t(ti) >= P.types.size()) fail(E_TYPECHECK, "unknown type");
    in = P.types[ti].params;
    out = P.types[ti].results;
  }

  void push_ctrl(CtrlKind k, std::vector<uint8_t> in, std::vector<uint8_t> out) {
    Ctrl c;
    c.kind = k;
    c.height = uint32_t(st.size() - in.size());
    c.cell_base = st.size() - in.size() < st.size() ? st[st.size() - in.size()].cell
                                                    : top_cell();
    if (in.empty()) c.cell_base = top_cell();
    c.in = std::move(in);
    c.out = std::move(out);
    c.dead = c.unreachable = !ctrl.empty() && ctrl.back().unreachable;
    ctrl.push_back(std::move(c));
  }

  const std::vector<uint8_t> &label_types(const Ctrl &c) const {
    return c.kind == C_LOOP ? c.in : c.out;
  }

  // Move the top `n` stack values into the canonical cells starting at dst_base.
  void move_top_to(size_t n, uint32_t dst_base) {
    uint32_t dst = dst_base;
    for (size_t k = st.size() - n; k < st.size(); k++) {
      materialize_into(st[k], dst);
      dst += cells_of(st[k].type);
    }
  }

  bool top_in_place(size_t n, uint32_t dst_base) const {
    uint32_t dst = dst_base;
    for (size_t k = st.size() - n; k < st.size(); k++) {
      if (st[k].kind != K_CELL || st[k].cell != dst) return false;
      dst += cells_of(st[k].type);
    }
    return true;
  }

  void branch_fixup(Ctrl &f, bool brtab, uint32_t index, int32_t extra) {
    if (f.label_known) {
      int32_t t = f.label_tcnt + extra;
      if (brtab) {
        P.brtab[2 * index] = f.label_pc;
        P.brtab[2 * index + 1] = uint32_t(t);
      } else {
        P.code[index].w3 = f.label_pc;
        P.code[index].w2 = (P.code[index].w2 & 0xFFFF) | (uint32_t(uint16_t(int16_t(t))) << 16);
      }
    } else {
      f.fixups.push_back(Fixup{brtab, index, extra});
    }
  }

  void resolve_label(Ctrl &f, uint32_t pc, int32_t tcnt) {
    f.label_known = true;
    f.label_pc = pc;
    f.label_tcnt = tcnt;
    for (const Fixup &x : f.fixups) {
      int32_t t = tcnt + x.extra;
      if (t < -32768 || t > 32767) fail(E_UNSUPPORTED, "tcnt overflow");
      if (x.brtab) {
        P.brtab[2 * x.index] = pc;
        P.brtab[2 * x.index + 1] = uint32_t(t);
      } else {
        P.code[x.index].w3 = pc;
        P.code[x.index].w2 = (P.code[x.index].w2 & 0xFFFF) | (uint32_t(uint16_t(int16_t(t))) << 16);
      }
    }
    f.fixups.clear();
  }

  void set_unreachable() {
    Ctrl &f = ctrl.back();
    st.resize(f.height);
    f.unreachable = true;
  }

  // retarget the last producer of the top entry to write `dst`; true on success
  bool try_retarget(const Entry &top, uint32_t dst) {
    if (!can_retarget || top.kind != K_CELL || top.producer < 0 || top.producer != last_emit)
      return false;
    DInstr &I = P.code[last_emit];
    if ((I.w2 & 0xFFFF) != top.cell) return false;
    uint32_t cnt = (I.w0 >> 16) & 0xFF, post = (I.w0 >> 24) & 0x7F;
    if (cnt + pending > 255 || post + pending > 127) return false;
    I.w2 = (I.w2 & 0xFFFF0000u) | dst;
    I.w0 = (I.w0 & (0xFFFFu | DBC_CTL)) | ((cnt + pending) << 16) | ((post + pending) << 24);
    pending = 0;
    take_pending(last_emit);
    return true;
  }

  // The instruction that produced stack entry `e` if it is the last one emitted, writes
  // e's canonical cell and no label intervened (so it can be merged with the consumer).
  DInstr *fusable_producer(const Entry &e, uint16_t op) {
    if (!can_retarget || e.kind != K_CELL || e.producer < 0 || e.producer != last_emit)
      return nullptr;
    DInstr &I = P.code[last_emit];
    if ((I.w0 & 0xFFFF) != op || (I.w2 & 0xFFFF) != e.cell) return nullptr;
    if (((I.w0 >> 16) & 0xFF) + pending > 255) return nullptr;
    return &I;
  }
  // merge the pending count into an already emitted instruction and retype it
  void fuse_into(DInstr &I, uint16_t op) {
    uint32_t cnt = ((I.w0 >> 16) & 0xFF) + pending;
    I.w0 = uint32_t(op) | (cnt << 16) | (is_ctl(op) ? DBC_CTL : 0u);
    pending = 0;
    take_pending(&I - P.code.data());
    if (cnt > P.max_wasm_instrs_per_dispatch) P.max_wasm_instrs_per_dispatch = cnt;
  }
  // the pending opcodes join an already emitted instruction's list (merged into it)
  void take_pending(int64_t pc) {
    auto &d = P.dops[size_t(pc)];
    d.insert(d.end(), pend_ops.begin(), pend_ops.end());
    pend_ops.clear();
  }
  void count_op(uint16_t op) { pending++; pend_ops.push_back(op); }
  void drop_pending() { pending = 0; pend_ops.clear(); }
  bool try_fuse_simple(const SimpleOp &s, Entry *ops);
  bool try_fuse_branch(const Entry &cond, bool branch_if_true, Ctrl &f);

  void do_simple(const SimpleOp &s);
  void do_load(uint16_t dop, uint8_t rtype, Reader &r);
  void do_store(uint16_t dop, uint8_t vtype, Reader &r);
  // MultiMemories (instruction.cpp:144-156, 374-389; formchecker.cpp:245-252)
  uint32_t nmems() const { return (P.has_mem ? 1u : 0u) + uint32_t(P.xmems.size()); }
  void check_mem(uint32_t k) {
    if (k >= nmems()) fail(P.multi_memory && nmems() ? 0x47 : E_TYPECHECK, "unknown memory");
  }
  // a memory-index immediate: a u32 with the proposal, else a zero byte
  uint32_t memidx(Reader &r) {
    if (P.multi_memory) return r.u32();
    if (r.u8() != 0) fail(E_TYPECHECK, "unknown memory");
    return 0;
  }
  // a memarg: align, offset, then (the proposal, align >= 64) the memory index
  uint32_t memarg(Reader &r, uint32_t *off) {
    const uint32_t al = r.u32();
    *off = r.u32();
    const uint32_t k = P.multi_memory && al >= 64 ? r.u32() : 0;
    check_mem(k);
    return k;
  }
  void do_call(uint32_t callee);
};

void Lowerer::do_simple(const SimpleOp &s) {
  const char *colon = strchr(s.sig, ':');
  int npop = int(colon - s.sig);
  Entry ops[3];
  for (int q = npop - 1; q >= 0; q--) ops[q] = pop_t(sigt(s.sig[q]));
  uint8_t rt = colon[1] ? sigt(colon[1]) : 0;
  bool var = false;
  for (int q = 0; q < npop; q++) var = var || ops[q].var;
  if (!live()) {
    if (rt) push_cell(rt);
    return;
  }
  if (try_fuse_simple(s, ops)) { push_cell(rt, last_emit).var = var; return; }
  uint32_t c = top_cell();  // result lands where the first operand was
  if (npop >= 1) c = ops[0].cell;
  if (npop == 2 && s.dop_imm >= 0) {
    int which = -1;
    if (ops[1].kind == K_CONST) which = 1;
    else if (s.commutative && ops[0].kind == K_CONST) which = 0;
    if (which >= 0) {
      bool fits = true;
      uint32_t imm = ops[which].k[0];
      if (ops[which].type == I64) {
        int64_t v = int64_t(uint64_t(ops[which].k[0]) | (uint64_t(ops[which].k[1]) << 32));
        fits = v >= INT32_MIN && v <= INT32_MAX;
      }
      if (fits) {
        uint32_t a = src(ops[1 - which]);
        emit(uint16_t(s.dop_imm), a, 0, c, 0, imm);
        push_cell(rt, last_emit).var = var;
        return;
      }
    }
  }
  uint32_t a = npop >= 1 ? src(ops[0]) : 0;
  uint32_t b = npop >= 2 ? src(ops[1]) : 0;
  uint32_t d = npop >= 3 ? src(ops[2]) : 0;
  emit(s.dop, a, b, c, d, s.imm);
  if (rt) push_cell(rt, last_emit).var = var;
}

// Superinstructions (merged into the previous DInstr; no label can intervene):
//   i32.add(i32.add(a, b), m)       -> I32_ADD3       (BLAKE3 G: a = a + b + m)
//   i32.rot{r,l}(i32.xor(a, b), k)  -> I32_XOR_ROT*_I (BLAKE3 G: d = rotr(d ^ a, k))
bool Lowerer::try_fuse_simple(const SimpleOp &s, Entry *ops) {
  if (s.dop == OP_I32_ADD) {
    for (int t = 0; t < 2; t++) {
      Entry &tmp = ops[t], &other = ops[1 - t];
      if (other.kind == K_CONST) continue;
      DInstr *I = fusable_producer(tmp, OP_I32_ADD);
      if (!I) continue;
      uint32_t oc = other.kind == K_LOCAL ? lcell[other.local] : other.cell;
      I->w2 = (I->w2 & 0xFFFF0000u) | ops[0].cell;      // result in the first operand's slot
      I->w2 = (I->w2 & 0xFFFFu) | (oc << 16);          // d = third addend
      fuse_into(*I, OP_I32_ADD3);
      return true;
    }
  }
  if ((s.dop == OP_I32_ROTR || s.dop == OP_I32_ROTL) && ops[1].kind == K_CONST) {
    DInstr *I = fusable_producer(ops[0], OP_I32_XOR);
    if (I) {
      I->w3 = ops[1].k[0];
      fuse_into(*I, s.dop == OP_I32_ROTR ? OP_I32_XOR_ROTR_I : OP_I32_XOR_ROTL_I);
      return true;
    }
  }
  return false;
}

// i32 compare feeding br_if / if -> one fused compare-and-branch (target/tcnt patched by
// the caller through the usual fixups). branch_if_true=false for `if` (branch when 0).
bool Lowerer::try_fuse_branch(const Entry &cond, bool branch_if_true, Ctrl &f) {
  (void)f;
  static const uint16_t cmp_rr[] = {OP_I32_EQ, OP_I32_NE, OP_I32_LT_S, OP_I32_LT_U, OP_I32_GT_S,
                                    OP_I32_GT_U, OP_I32_LE_S, OP_I32_LE_U, OP_I32_GE_S, OP_I32_GE_U};
  // negation: eq<->ne, lt_s<->ge_s, lt_u<->ge_u, gt_s<->le_s, gt_u<->le_u
  static const int neg[] = {1, 0, 8, 9, 6, 7, 4, 5, 2, 3};
  if (!can_retarget || cond.kind != K_CELL || cond.producer < 0 || cond.producer != last_emit)
    return false;
  DInstr &I = P.code[last_emit];
  uint16_t op = I.w0 & 0xFFFF;
  if ((I.w2 & 0xFFFF) != cond.cell) return false;
  if (((I.w0 >> 16) & 0xFF) + pending > 255) return false;
  if (op == OP_I32_EQZ) {      // eqz + br_if -> BR_UNLESS ; eqz + if -> BR_IF
    I.w2 = 0;
    fuse_into(I, branch_if_true ? OP_BR_UNLESS : OP_BR_IF);
    return true;
  }
  for (int k = 0; k < 10; k++) {
    int kk = branch_if_true ? k : neg[k];
    if (op == cmp_rr[k]) {
      I.w2 = 0;
      fuse_into(I, uint16_t(OP_BR_EQ + kk));
      return true;
    }
    if (op == cmp_rr[k] - OP_I32_ADD + OP_I32_ADD_I) {
      int32_t v = int32_t(I.w3);
      if (v < -32768 || v > 32767) return false;
      I.w1 = (I.w1 & 0xFFFF) | (uint32_t(uint16_t(int16_t(v))) << 16);
      I.w2 = 0;
      I.w3 = 0;
      fuse_into(I, uint16_t(OP_BR_EQ_I + kk));
      return true;
    }
  }
  return false;
}

void Lowerer::do_load(uint16_t dop, uint8_t rtype, Reader &r) {
  uint32_t off;
  const uint32_t k = memarg(r, &off);
  Entry a = pop_t(I32);
  if (a.var) (k ? P.divergent_xmem : P.divergent_mem) = true;
  if (!live()) { push_cell(rtype); return; }
  uint32_t ac = src(a);
  if (k) emit(OP_XLD, ac, k, a.cell, dop, off);   // (memory k: compiled runs, else the per-lane step)
  else emit(dop, ac, 0, a.cell, 0, off);
  push_cell(rtype, last_emit);
}

void Lowerer::do_store(uint16_t dop, uint8_t vtype, Reader &r) {
  uint32_t off;
  const uint32_t k = memarg(r, &off);
  Entry v = pop_t(vtype);
  Entry a = pop_t(I32);
  if (a.var) (k ? P.divergent_xmem : P.divergent_mem) = true;
  if (!live()) return;
  uint32_t ac = src(a), vc = src(v);
  if (k) emit(OP_XST, ac, vc, k, dop, off);
  else emit(dop, ac, vc, 0, 0, off);
}

void Lowerer::do_call(uint32_t callee) {
  if (callee >= P.funcs.size()) fail(E_TYPECHECK, "unknown function");
  const FuncType &t = P.types[P.funcs[callee].type];
  size_t np = t.params.size();
  // type-check args
  std::vector<Entry> args(np);
  for (size_t k = np; k > 0; k--) args[k - 1] = pop_t(t.params[k - 1]);
  if (!P.funcs[callee].imported)
    for (size_t k = 0; k < np; k++)
      if (args[k].var) set_var_local(callee, uint32_t(k));
  if (!live()) {
    for (uint8_t r : t.results) push_cell(r);
    return;
  }
  for (auto &e : args) st.push_back(e);
  materialize_top(np);
  uint32_t argcells = 0;
  for (auto &e : args) argcells += cells_of(e.type);
  uint32_t L = top_cell() - argcells;
  st.resize(st.size() - np);
  if (P.funcs[callee].imported) {   // helper.cpp:35-97: runs on the CPU executor
    uint32_t rc = 0;
    for (uint8_t r : t.results) rc += cells_of(r);
    emit(OP_HOST_CALL, L, argcells, rc, 0, callee);
  } else {
    uint32_t rc = 0;
    for (uint8_t r : t.results) rc += cells_of(r);
    emit(OP_CALL, L, argcells, P.funcs[callee].local_cells, 0, 0);
    callfix->push_back(CallFix{uint32_t(last_emit), callee});
    emit(OP_POST_CALL, L, rc);
  }
  for (uint8_t r : t.results) push_cell(r);
  uint32_t hi = L + argcells;
  if (hi > max_cell) max_cell = hi;
}


// ------------------------------------------------------------------ lower one function
void Lowerer::lower_function(uint32_t fi, std::vector<CallFix> &cf) {
  callfix = &cf;
  cur_fn = fi;
  FuncInfo &F = P.funcs[fi];
  ft = &P.types[F.type];
  ltypes = ft->params;
  ltypes.insert(ltypes.end(), F.local_types.begin(), F.local_types.end());
  frame_base = P.global_cells;
  lcell.clear();
  uint32_t cc = frame_base;
  for (uint8_t t : ltypes) { lcell.push_back(cc); cc += cells_of(t); }
  F.param_cells = 0;
  for (uint8_t t : ft->params) F.param_cells += cells_of(t);
  F.local_cells = cc - frame_base - F.param_cells;
  opnd_base = cc;
  max_cell = cc;
  st.clear();
  ctrl.clear();
  drop_pending();
  last_emit = -1;
  can_retarget = false;

  F.entry_pc = uint32_t(P.code.size());
  if (F.local_cells) {   // prologue used by call_indirect / the kernel's first frame
    P.code.push_back(DInstr{OP_ZERO_LOCALS, (frame_base + F.param_cells) | (F.local_cells << 16), 0, 0});
    P.dops.emplace_back();
  }
  F.body_pc = uint32_t(P.code.size());
  push_ctrl(C_FUNC, {}, ft->results);

  Reader r{bin + F.code_off, bin + F.code_off + F.code_len};
  const auto &simple = simple_ops();
  while (!ctrl.empty()) {
    uint16_t op = r.u8();
    if (op == 0xFC || op == 0xFD) {
      uint32_t sub = r.u32();
      if (sub > 0xFF) fail(E_ILLEGAL_OPCODE, "illegal opcode");
      op = uint16_t(op << 8 | sub);
    }
    if (op != 0x0B && op != 0x05 && op != 0x03) count_op(op);  // else/end/loop: at their labels
    auto it = simple.find(op);
    if (it != simple.end()) { do_simple(it->second); continue; }
    switch (op) {
      case 0x00:  // unreachable (engine.cpp:79-83)
        if (live()) emit(OP_UNREACHABLE, 0, 0, 0, 0, 0x89);
        set_unreachable();
        break;
      case 0x01: break;  // nop: counted, folded
      case 0x02: case 0x03: case 0x04: {
        std::vector<uint8_t> in, out;
        block_type(r, in, out);
        Entry cond{};
        if (op == 0x04) cond = pop_t(I32);
        std::vector<Entry> ps(in.size());
        for (size_t k = in.size(); k > 0; k--) ps[k - 1] = pop_t(in[k - 1]);
        for (auto &e : ps) st.push_back(e);
        if (live()) {           // locals may change inside: no lazy local refs across
          materialize_locals();
          materialize_top(in.size());
        }
        if (op == 0x02) {
          push_ctrl(C_BLOCK, in, out);
        } else if (op == 0x03) {
          // br to a loop lands on (and re-counts) the `loop` instruction
          place_label();
          int32_t tcnt = -int32_t(pending);
          uint32_t lpc = uint32_t(P.code.size());
          count_op(0x03);
          push_ctrl(C_LOOP, in, out);
          if (!ctrl.back().dead) resolve_label(ctrl.back(), lpc, tcnt);
        } else {
          int64_t br = -1;
          if (live()) {
            if (in.empty() && try_fuse_branch(cond, false, ctrl.back())) {
              br = last_emit;
            } else {
              uint32_t c;
              if (cond.kind == K_LOCAL) c = lcell[cond.local];
              else {
                if (cond.kind == K_CONST) materialize_into(cond, cond.cell);
                c = cond.cell;
              }
              emit(OP_BR_UNLESS, c, 0, 0, 0, 0);
              br = last_emit;
            }
          }
          push_ctrl(C_IF, in, out);
          ctrl.back().else_br = br;
        }
        break;
      }
      case 0x05: {  // else (controlInstr.cpp:11-34, engine.cpp:92-110)
        Ctrl &f = ctrl.back();
        if (f.kind != C_IF || f.has_else) fail(E_ILLEGAL_OPCODE, "else outside if");
        if (!f.unreachable) {
          std::vector<Entry> vals(f.out.size());
          for (size_t k = f.out.size(); k > 0; k--) vals[k - 1] = pop_t(f.out[k - 1]);
          if (st.size() != f.height) fail(E_TYPECHECK, "type mismatch at else");
          for (auto &e : vals) st.push_back(e);
          move_top_to(f.out.size(), f.cell_base);
          count_op(0x05);                   // the `else` dispatch on the then-path
          emit(OP_JMP);
          branch_fixup(f, false, uint32_t(last_emit), -1);  // end is not re-counted
        } else {
          drop_pending();
        }
        st.resize(f.height);
        for (uint8_t t : f.in) push_cell(t);
        f.unreachable = f.dead;
        place_label();
        if (f.else_br >= 0) {               // if-false path: counts `else` manually (+1)
          P.code[f.else_br].w3 = uint32_t(P.code.size());
          P.code[f.else_br].w2 = (P.code[f.else_br].w2 & 0xFFFF) | (1u << 16);
          f.else_br = -1;
        }
        f.has_else = true;
        break;
      }
      case 0x0B: {  // end
        Ctrl &f = ctrl.back();
        if (!f.unreachable) {
          std::vector<Entry> vals(f.out.size());
          for (size_t k = f.out.size(); k > 0; k--) vals[k - 1] = pop_t(f.out[k - 1]);
          if (st.size() != f.height) fail(E_TYPECHECK, "type mismatch at end");
          for (auto &e : vals) st.push_back(e);
          move_top_to(f.out.size(), f.cell_base);
        } else {
          drop_pending();
        }
        if (f.kind == C_IF && !f.has_else) {
          if (f.in != f.out) fail(E_TYPECHECK, "if without else must not change the stack");
          if (f.else_br >= 0) branch_fixup(f, false, uint32_t(f.else_br), 0);
        }
        place_label();
        int32_t tcnt = -int32_t(pending);
        uint32_t lpc = uint32_t(P.code.size());
        count_op(0x0B);                     // the `end` itself
        if (f.kind != C_LOOP && !f.dead) resolve_label(f, lpc, tcnt);
        if (f.kind == C_FUNC) {
          uint32_t rc = 0;
          for (uint8_t t : f.out) rc += cells_of(t);
          emit(OP_RET, opnd_base, rc);
          ctrl.pop_back();
          break;
        }
        Ctrl done = std::move(ctrl.back());
        ctrl.pop_back();
        st.resize(done.height);
        for (uint8_t t : done.out) push_cell(t);
        break;
      }
      case 0x0C: case 0x0D: {  // br / br_if (controlInstr.cpp:36-51, helper.cpp:179-193)
        uint32_t depth = r.u32();
        if (depth >= ctrl.size()) fail(E_TYPECHECK, "unknown label");
        Entry cond{};
        if (op == 0x0D) cond = pop_t(I32);
        Ctrl &f = ctrl[ctrl.size() - 1 - depth];
        const std::vector<uint8_t> lt = label_types(f);
        std::vector<Entry> vals(lt.size());
        for (size_t k = lt.size(); k > 0; k--) vals[k - 1] = pop_t(lt[k - 1]);
        for (auto &e : vals) st.push_back(e);
        if (!live()) { if (op == 0x0C) set_unreachable(); break; }
        size_t n = lt.size();
        if (op == 0x0C) {
          move_top_to(n, f.cell_base);
          emit(OP_JMP);
          branch_fixup(f, false, uint32_t(last_emit), 0);
          set_unreachable();
          break;
        }
        uint32_t c;
        if (cond.kind == K_LOCAL) c = lcell[cond.local];
        else {
          if (cond.kind == K_CONST) materialize_into(cond, cond.cell);
          c = cond.cell;
        }
        if (n == 0 || top_in_place(n, f.cell_base)) {
          if (!try_fuse_branch(cond, true, f)) emit(OP_BR_IF, c);
          branch_fixup(f, false, uint32_t(last_emit), 0);
        } else if (n == 1 && cells_of(st.back().type) <= 2) {
          Entry &e = st.back();
          if (e.kind == K_CONST) materialize(st.size() - 1);
          uint32_t s = e.kind == K_LOCAL ? lcell[e.local] : e.cell;
          emit(cells_of(e.type) == 1 ? OP_BR_IF_MOV1 : OP_BR_IF_MOV2, c, s, f.cell_base);
          branch_fixup(f, false, uint32_t(last_emit), 0);
        } else {
          emit(OP_BR_UNLESS, c);
          uint32_t skip = uint32_t(last_emit);
          move_top_to(n, f.cell_base);
          emit(OP_JMP);
          branch_fixup(f, false, uint32_t(last_emit), 0);
          place_label();
          P.code[skip].w3 = uint32_t(P.code.size());
        }
        break;
      }
      case 0x0E: {  // br_table (controlInstr.cpp:53-70)
        uint32_t n = r.u32();
        std::vector<uint32_t> depths(n + 1);
        for (uint32_t k = 0; k <= n; k++) {
          depths[k] = r.u32();
          if (depths[k] >= ctrl.size()) fail(E_TYPECHECK, "unknown label");
        }
        Entry idx = pop_t(I32);
        const std::vector<uint8_t> lt = label_types(ctrl[ctrl.size() - 1 - depths[n]]);
        for (uint32_t k = 0; k < n; k++)
          if (label_types(ctrl[ctrl.size() - 1 - depths[k]]).size() != lt.size())
            fail(E_TYPECHECK, "br_table arity mismatch");
        std::vector<Entry> vals(lt.size());
        for (size_t k = lt.size(); k > 0; k--) vals[k - 1] = pop_t(lt[k - 1]);
        for (auto &e : vals) st.push_back(e);
        if (live()) {
          uint32_t ic = src(idx);
          uint32_t base = uint32_t(P.brtab.size() / 2);
          P.brtab.resize(P.brtab.size() + 2 * (n + 1), 0);
          emit(OP_BR_TABLE, ic, n, 0, 0, base);
          for (uint32_t k = 0; k <= n; k++) {
            Ctrl &f = ctrl[ctrl.size() - 1 - depths[k]];
            if (lt.empty() || top_in_place(lt.size(), f.cell_base)) {
              branch_fixup(f, true, base + k, 0);
            } else {                       // trampoline: move values, jump
              place_label();
              P.brtab[2 * (base + k)] = uint32_t(P.code.size());
              P.brtab[2 * (base + k) + 1] = 0;
              move_top_to(lt.size(), f.cell_base);
              emit(OP_JMP);
              branch_fixup(f, false, uint32_t(last_emit), 0);
            }
          }
        }
        set_unreachable();
        break;
      }
      case 0x0F: {  // return (controlInstr.cpp:72-81): the function `end` is not counted
        std::vector<Entry> vals(ft->results.size());
        for (size_t k = ft->results.size(); k > 0; k--) vals[k - 1] = pop_t(ft->results[k - 1]);
        if (live()) {
          for (auto &e : vals) st.push_back(e);
          materialize_top(vals.size());
          uint32_t rc = 0;
          for (auto &e : vals) rc += cells_of(e.type);
          emit(OP_RET, top_cell() - rc, rc);
        }
        set_unreachable();
        break;
      }
      case 0x10: do_call(r.u32()); break;
      case 0x11: {  // call_indirect (controlInstr.cpp:101-158)
        uint32_t ti = r.u32();
        uint32_t tab = r.u32();
        if (ti >= P.types.size() || tab >= P.ntables) fail(E_TYPECHECK, "unknown type/table");
        if (P.tables[tab].type != FUNCREF) fail(E_TYPECHECK, "type mismatch");
        Entry idx = pop_t(I32);
        const FuncType &t = P.types[ti];
        std::vector<Entry> args(t.params.size());
        for (size_t k = args.size(); k > 0; k--) args[k - 1] = pop_t(t.params[k - 1]);
        if (live()) {
          for (auto &e : args) st.push_back(e);
          materialize_top(args.size());
          uint32_t argcells = 0;
          for (auto &e : args) argcells += cells_of(e.type);
          uint32_t L = top_cell() - argcells;
          uint32_t ic = src(idx);
          if (ic + 1 > max_cell) max_cell = ic + 1;
          st.resize(st.size() - args.size());
          uint32_t rc = 0;
          for (uint8_t r : t.results) rc += cells_of(r);
          emit(OP_CALL_INDIRECT, L, argcells, ic, tab, P.type_canon[ti]);
          emit(OP_POST_CALL, L, rc);
        }
        for (uint8_t rt : t.results) push_cell(rt);
        break;
      }
      case 0x12: case 0x13: {  // return_call / return_call_indirect (TailCall proposal;
                               // formchecker.cpp:515-560, controlInstr.cpp:83-158)
        if (!P.tail_call) fail(E_ILLEGAL_OPCODE, "return_call needs the TailCall proposal");
        const bool ind = op == 0x13;
        uint32_t callee = 0, ti = 0, tab = 0;
        if (ind) {
          ti = r.u32();
          tab = r.u32();
          if (tab >= P.ntables || P.tables[tab].type != FUNCREF) fail(E_TYPECHECK, "unknown table");
          if (ti >= P.types.size()) fail(E_TYPECHECK, "unknown type");
        } else {
          callee = r.u32();
          if (callee >= P.funcs.size()) fail(E_TYPECHECK, "unknown function");
          ti = P.funcs[callee].type;
        }
        const FuncType &t = P.types[ti];
        if (t.results != ft->results) fail(E_TYPECHECK, "type mismatch");   // the caller's results
        Entry idx{};
        if (ind) idx = pop_t(I32);
        std::vector<Entry> args(t.params.size());
        for (size_t k = args.size(); k > 0; k--) args[k - 1] = pop_t(t.params[k - 1]);
        if (!ind && !P.funcs[callee].imported)
          for (size_t k = 0; k < args.size(); k++)
            if (args[k].var) set_var_local(callee, uint32_t(k));
        if (live()) {
          for (auto &e : args) st.push_back(e);
          materialize_top(args.size());
          uint32_t argcells = 0;
          for (auto &e : args) argcells += cells_of(e.type);
          const uint32_t L = top_cell() - argcells;
          uint32_t ic = 0;
          if (ind) {
            ic = src(idx);
            if (ic + 1 > max_cell) max_cell = ic + 1;
          }
          st.resize(st.size() - args.size());
          uint32_t rc = 0;
          for (uint8_t rt : t.results) rc += cells_of(rt);
          // A host import called in tail position runs in the caller's reused frame, which
          // it then pops (helper.cpp:35-97 with IsTailCall, stackmgr.h:80-112): its results
          // leave like a `return`. The reference resumes at the frame's From, which a
          // native frame stores one instruction early (helper.cpp:163, RetIt - 1): from the
          // entry function that re-executes the function's final `end` (counted and priced,
          // then the run ends with the host's results), so the RET here retires one `end`.
          // (From a nested frame the reference would re-execute its caller's call
          // instruction instead; this returns to the caller -- DESIGN.md "Tail calls".)
          // return_call_indirect may reach a host import at run time: its RET follows it,
          // reached only then (dbc_step.inc).
          auto host_ret = [&]() {
            pending += 1;
            pend_ops.push_back(0x0B);
            emit(OP_RET, L, rc);
          };
          if (ind) {
            emit(OP_TAIL_CALL_INDIRECT, L, argcells, ic, tab, P.type_canon[ti]);
            host_ret();
          } else if (P.funcs[callee].imported) {
            emit(OP_HOST_CALL, L, argcells, rc, 0, callee);
            host_ret();
          } else {
            emit(OP_TAIL_CALL, L, argcells, P.funcs[callee].local_cells, 0, 0);
            callfix->push_back(CallFix{uint32_t(last_emit), callee});
          }
          if (L + argcells > max_cell) max_cell = L + argcells;
        }
        set_unreachable();
        break;
      }
      case 0x1A: pop_any(); break;  // drop
      case 0x1B: case 0x1C: {       // select (engine.cpp:152-166)
        uint8_t want = UNKNOWN;
        if (op == 0x1C) {
          uint32_t n = r.u32();
          if (n != 1) fail(E_TYPECHECK, "invalid result arity");
          want = r.u8();
        }
        Entry cnd = pop_t(I32);
        Entry v2 = pop_t(want), v1 = pop_t(want);
        if (v1.type != v2.type && v1.type != UNKNOWN && v2.type != UNKNOWN)
          fail(E_TYPECHECK, "type mismatch");
        uint8_t t = v1.type != UNKNOWN ? v1.type : v2.type;
        if (!live()) { push_cell(t == UNKNOWN ? I32 : t); break; }
        uint32_t w = cells_of(t);
        uint32_t a = src(v1), b = src(v2), d = src(cnd);
        emit(w == 1 ? OP_SELECT32 : w == 2 ? OP_SELECT64 : OP_SELECT128, a, b, v1.cell, d);
        push_cell(t, last_emit);
        break;
      }
      case 0x20: {  // local.get (variableInstr.cpp:11-15): a lazy reference
        uint32_t li = r.u32();
        if (li >= ltypes.size()) fail(E_TYPECHECK, "unknown local");
        push_local(li);
        break;
      }
      case 0x21: case 0x22: {  // local.set / local.tee (variableInstr.cpp:17-30)
        uint32_t li = r.u32();
        if (li >= ltypes.size()) fail(E_TYPECHECK, "unknown local");
        Entry v = pop_t(ltypes[li]);
        if (v.var) set_var_local(cur_fn, li);
        if (!live()) { if (op == 0x22) push_cell(ltypes[li]); break; }
        if (v.kind == K_LOCAL && v.local == li) { if (op == 0x22) st.push_back(v); break; }
        materialize_locals(li);
        if (try_retarget(v, lcell[li])) {
          if (op == 0x22) push_local(li);
        } else {
          materialize_into(v, lcell[li]);
          if (op == 0x22) st.push_back(v);
        }
        break;
      }
      case 0x23: case 0x24: {  // global.get / global.set (variableInstr.cpp:32-44)
        uint32_t gi = r.u32();
        if (gi >= P.global_types.size()) fail(E_TYPECHECK, "unknown global");
        uint8_t t = P.global_types[gi];
        uint32_t w = cells_of(t);
        if (op == 0x23) {
          if (live()) {
            uint32_t dst = top_cell();
            emit(w == 1 ? OP_MOV32 : w == 2 ? OP_MOV64 : OP_MOV128, P.global_cell[gi], 0, dst);
            push_cell(t, last_emit).var = P.global_mut[gi] != 0;   // a constant global is uniform
          } else push_cell(t);
        } else {
          if (!P.global_mut[gi]) fail(E_TYPECHECK, "global is immutable");
          Entry v = pop_t(t);
          if (!live()) break;
          if (P.exact_globals || !try_retarget(v, P.global_cell[gi]))
            materialize_into(v, P.global_cell[gi]);
        }
        break;
      }
      case 0x25: {  // table.get (tableInstr.cpp; shared table 0 or the lane's own table)
        uint32_t tab = r.u32();
        if (tab >= P.ntables) fail(E_TYPECHECK, "unknown table");
        const uint8_t rt = P.tables[tab].type;
        Entry idx = pop_t(I32);
        if (!live()) { push_cell(rt); break; }
        uint32_t ic = src(idx);
        emit(OP_TABLE_GET, ic, 0, idx.cell, tab);
        push_cell(rt, last_emit);
        break;
      }
      case 0x26: {  // table.set
        uint32_t tab = r.u32();
        if (tab >= P.ntables) fail(E_TYPECHECK, "unknown table");
        need_mut_tables();
        Entry v = pop_t(P.tables[tab].type), idx = pop_t(I32);
        if (!live()) break;
        uint32_t ic = src(idx), vc = src(v);
        emit(OP_TABLE_SET, ic, vc, 0, tab);
        break;
      }
      // ---- memory (memory.ipp:12-68)
      case 0x28: do_load(OP_LD32, I32, r); break;
      case 0x29: do_load(OP_LD64, I64, r); break;
      case 0x2A: do_load(OP_LD32, F32, r); break;
      case 0x2B: do_load(OP_LD64, F64, r); break;
      case 0x2C: do_load(OP_LD8S32, I32, r); break;
      case 0x2D: do_load(OP_LD8U32, I32, r); break;
      case 0x2E: do_load(OP_LD16S32, I32, r); break;
      case 0x2F: do_load(OP_LD16U32, I32, r); break;
      case 0x30: do_load(OP_LD8S64, I64, r); break;
      case 0x31: do_load(OP_LD8U64, I64, r); break;
      case 0x32: do_load(OP_LD16S64, I64, r); break;
      case 0x33: do_load(OP_LD16U64, I64, r); break;
      case 0x34: do_load(OP_LD32S64, I64, r); break;
      case 0x35: do_load(OP_LD32U64, I64, r); break;
      case 0x36: do_store(OP_ST32, I32, r); break;
      case 0x37: do_store(OP_ST64, I64, r); break;
      case 0x38: do_store(OP_ST32, F32, r); break;
      case 0x39: do_store(OP_ST64, F64, r); break;
      case 0x3A: do_store(OP_ST8, I32, r); break;
      case 0x3B: do_store(OP_ST16, I32, r); break;
      case 0x3C: do_store(OP_ST8, I64, r); break;
      case 0x3D: do_store(OP_ST16, I64, r); break;
      case 0x3E: do_store(OP_ST32, I64, r); break;
      case 0x3F: {  // memory.size (memoryInstr.cpp:9-15)
        const uint32_t k = memidx(r);
        check_mem(k);
        if (live()) {
          if (k) emit(OP_XMEM_SIZE, 0, k, top_cell());
          else emit(OP_MEM_SIZE, 0, 0, top_cell());
          push_cell(I32, last_emit);
        } else {
          push_cell(I32);
        }
        break;
      }
      case 0x40: {  // memory.grow (memoryInstr.cpp:17-31)
        const uint32_t k = memidx(r);
        check_mem(k);
        Entry n = pop_t(I32);
        if (!live()) { push_cell(I32); break; }
        uint32_t a = src(n);
        if (k) emit(OP_XMEM_GROW, a, k, n.cell);
        else emit(OP_MEM_GROW, a, 0, n.cell);
        push_cell(I32, last_emit);
        break;
      }
      case 0x41: { uint32_t k[4] = {uint32_t(int32_t(r.sleb(32))), 0, 0, 0}; push_const(I32, k); break; }
      case 0x42: { uint64_t v = uint64_t(r.sleb(64)); uint32_t k[4] = {uint32_t(v), uint32_t(v >> 32), 0, 0}; push_const(I64, k); break; }
      case 0x43: { uint32_t k[4] = {0, 0, 0, 0}; for (int q = 0; q < 4; q++) k[0] |= uint32_t(r.u8()) << (8 * q); push_const(F32, k); break; }
      case 0x44: { uint64_t v = 0; for (int q = 0; q < 8; q++) v |= uint64_t(r.u8()) << (8 * q);
                   uint32_t k[4] = {uint32_t(v), uint32_t(v >> 32), 0, 0}; push_const(F64, k); break; }
      case 0xA7: {  // i32.wrap_i64: the low cell of an i64 slot already is the i32
        Entry v = pop_t(I64);
        if (!live()) { push_cell(I32); break; }
        if (v.kind == K_CONST) { uint32_t k[4] = {v.k[0], 0, 0, 0}; push_const(I32, k); }
        else if (v.kind == K_LOCAL) { emit(OP_MOV32, lcell[v.local], 0, v.cell); push_cell(I32, last_emit); }
        else push_cell(I32);
        break;
      }
      case 0xBC: case 0xBD: case 0xBE: case 0xBF: {  // reinterpret: same bits, retype
        static const uint8_t from[] = {F32, F64, I32, I64}, to[] = {I32, I64, F32, F64};
        Entry v = pop_t(from[op - 0xBC]);
        v.type = to[op - 0xBC];
        if (v.kind == K_LOCAL) {  // keep lazily, but the entry's type differs from the local's
          if (live()) { emit(cells_of(v.type) == 1 ? OP_MOV32 : OP_MOV64, lcell[v.local], 0, v.cell); }
          v.kind = K_CELL;
          v.producer = live() ? last_emit : -1;
        }
        st.push_back(v);
        break;
      }
      case 0xD0: { uint8_t t = r.u8(); uint32_t k[4] = {0xFFFFFFFFu, 0, 0, 0}; push_const(t, k); break; }
      case 0xD1: {  // ref.is_null
        Entry v = pop_any();
        if (v.type != FUNCREF && v.type != EXTERNREF && v.type != UNKNOWN) fail(E_TYPECHECK, "type mismatch");
        if (!live()) { push_cell(I32); break; }
        uint32_t a = src(v);
        emit(OP_I32_EQ_I, a, 0, v.cell, 0, 0xFFFFFFFFu);
        push_cell(I32, last_emit);
        break;
      }
      case 0xD2: { uint32_t f = r.u32(); if (f >= P.funcs.size()) fail(E_TYPECHECK, "unknown function");
                   uint32_t k[4] = {f, 0, 0, 0}; push_const(FUNCREF, k); break; }
      case 0xFC08: {  // memory.init (memoryInstr.cpp:33-49)
        uint32_t di = r.u32();
        const uint32_t k = memidx(r);
        check_mem(k);   // (the memory first, formchecker.cpp:812-824)
        if (di >= P.datas.size()) fail(P.multi_memory ? 0x4A : E_TYPECHECK, "unknown data");
        Entry n = pop_t(I32), s = pop_t(I32), d = pop_t(I32);
        if (!live()) break;
        uint32_t dc = src(d), sc = src(s), nc = src(n);
        if (k) emit(OP_XMEM_INIT, dc, sc, nc, k, di);
        else emit(OP_MEM_INIT, dc, sc, nc, 0, di);
        break;
      }
      case 0xFC09: {
        uint32_t di = r.u32();
        if (di >= P.datas.size()) fail(E_TYPECHECK, "unknown data");
        if (live()) emit(OP_DATA_DROP, 0, 0, 0, 0, di);
        break;
      }
      case 0xFC0A: case 0xFC0B: {  // memory.copy / memory.fill (memoryInstr.cpp:59-101)
        const uint32_t k = memidx(r), k2 = op == 0xFC0A ? memidx(r) : 0;
        if (op == 0xFC0A) check_mem(k2);   // (copy: the source first, formchecker.cpp:826-834)
        check_mem(k);
        Entry n = pop_t(I32), s = pop_t(I32), d = pop_t(I32);
        if (!live()) break;
        uint32_t dc = src(d), sc = src(s), nc = src(n);
        if (op == 0xFC0A && (k || k2)) emit(OP_XMEM_COPY, dc, sc, nc, 0, k | (k2 << 16));
        else if (op == 0xFC0B && k) emit(OP_XMEM_FILL, dc, sc, nc, 0, k);
        else emit(op == 0xFC0A ? OP_MEM_COPY : OP_MEM_FILL, dc, sc, nc);
        break;
      }
      case 0xFC10: {  // table.size: a constant for the shared immutable table
        uint32_t tab = r.u32();
        if (tab >= P.ntables) fail(E_TYPECHECK, "unknown table");
        if (!P.mut_tables) {
          uint32_t k[4] = {uint32_t(P.table0.size()), 0, 0, 0};
          push_const(I32, k);
        } else if (live()) {
          emit(OP_TABLE_SIZE, 0, 0, top_cell(), tab);
          push_cell(I32, last_emit);
        } else {
          push_cell(I32);
        }
        break;
      }
      case 0xFC0C: {  // table.init elem table (tableInstr.cpp)
        uint32_t ei = r.u32(), tab = r.u32();
        if (tab >= P.ntables || ei >= P.elems.size()) fail(E_TYPECHECK, "unknown table/elem");
        if (P.elems[ei].type != P.tables[tab].type) fail(E_TYPECHECK, "type mismatch");
        need_mut_tables();
        Entry n = pop_t(I32), sidx = pop_t(I32), d = pop_t(I32);
        if (!live()) break;
        uint32_t dc = src(d), sc = src(sidx), nc = src(n);
        emit(OP_TABLE_INIT, dc, sc, nc, 0, tab | (ei << 16));
        break;
      }
      case 0xFC0D: {  // elem.drop
        uint32_t ei = r.u32();
        if (ei >= P.elems.size()) fail(E_TYPECHECK, "unknown elem");
        need_mut_tables();
        if (live()) emit(OP_ELEM_DROP, 0, 0, 0, 0, ei);
        break;
      }
      case 0xFC0E: {  // table.copy dst src
        uint32_t td = r.u32(), ts = r.u32();
        if (td >= P.ntables || ts >= P.ntables) fail(E_TYPECHECK, "unknown table");
        if (P.tables[td].type != P.tables[ts].type) fail(E_TYPECHECK, "type mismatch");
        need_mut_tables();
        Entry n = pop_t(I32), sidx = pop_t(I32), d = pop_t(I32);
        if (!live()) break;
        uint32_t dc = src(d), sc = src(sidx), nc = src(n);
        emit(OP_TABLE_COPY, dc, sc, nc, 0, td | (ts << 16));
        break;
      }
      case 0xFC0F: {  // table.grow
        uint32_t tab = r.u32();
        if (tab >= P.ntables) fail(E_TYPECHECK, "unknown table");
        need_mut_tables();
        Entry n = pop_t(I32), v = pop_t(P.tables[tab].type);
        if (!live()) { push_cell(I32); break; }
        uint32_t vc = src(v), nc = src(n);
        emit(OP_TABLE_GROW, vc, nc, v.cell, tab);
        push_cell(I32, last_emit);
        break;
      }
      case 0xFC11: {  // table.fill
        uint32_t tab = r.u32();
        if (tab >= P.ntables) fail(E_TYPECHECK, "unknown table");
        need_mut_tables();
        Entry n = pop_t(I32), v = pop_t(P.tables[tab].type), d = pop_t(I32);
        if (!live()) break;
        uint32_t dc = src(d), vc = src(v), nc = src(n);
        emit(OP_TABLE_FILL, dc, vc, nc, 0, tab);
        break;
      }
      // ---- SIMD memory
      case 0xFD00: do_load(OP_LD128, V128, r); break;
      case 0xFD01: do_load(OP_V_LD8X8S, V128, r); break;
      case 0xFD02: do_load(OP_V_LD8X8U, V128, r); break;
      case 0xFD03: do_load(OP_V_LD16X4S, V128, r); break;
      case 0xFD04: do_load(OP_V_LD16X4U, V128, r); break;
      case 0xFD05: do_load(OP_V_LD32X2S, V128, r); break;
      case 0xFD06: do_load(OP_V_LD32X2U, V128, r); break;
      case 0xFD07: do_load(OP_V_LD8SPLAT, V128, r); break;
      case 0xFD08: do_load(OP_V_LD16SPLAT, V128, r); break;
      case 0xFD09: do_load(OP_V_LD32SPLAT, V128, r); break;
      case 0xFD0A: do_load(OP_V_LD64SPLAT, V128, r); break;
      case 0xFD5C: do_load(OP_V_LD32ZERO, V128, r); break;
      case 0xFD5D: do_load(OP_V_LD64ZERO, V128, r); break;
      case 0xFD0B: do_store(OP_ST128, V128, r); break;
      case 0xFD54: case 0xFD55: case 0xFD56: case 0xFD57:     // v128.loadN_lane
      case 0xFD58: case 0xFD59: case 0xFD5A: case 0xFD5B: {   // v128.storeN_lane
        const bool ld = op <= 0xFD57;
        const uint32_t lg = (op - 0xFD54) & 3;                 // log2 of the lane bytes
        uint32_t off;
        const uint32_t k = memarg(r, &off);
        uint8_t lane = r.u8();
        if (lane >= (16u >> lg)) fail(E_TYPECHECK, "invalid lane index");
        Entry v = pop_t(V128), a = pop_t(I32);
        if (!live()) { if (ld) push_cell(V128); break; }
        uint32_t ac = src(a), vc = src(v);
        if (k) emit(OP_XLANE, ac, vc, ld ? a.cell : 0, lane | (lg << 4) | (ld ? 64u : 0u) | (k << 8), off);
        else emit(ld ? OP_V_LDLANE : OP_V_STLANE, ac, vc, ld ? a.cell : 0, lane | (lg << 8), off);
        if (ld) push_cell(V128, last_emit);
        break;
      }
      case 0xFD0C: {
        uint32_t k[4];
        for (int q = 0; q < 4; q++) {
          k[q] = 0;
          for (int b = 0; b < 4; b++) k[q] |= uint32_t(r.u8()) << (8 * b);
        }
        push_const(V128, k);
        break;
      }
      case 0xFD0D: {  // i8x16.shuffle: mask in the v128 pool
        uint32_t k[4];
        for (int q = 0; q < 4; q++) {
          k[q] = 0;
          for (int b = 0; b < 4; b++) {
            uint8_t lane = r.u8();
            if (lane >= 32) fail(E_TYPECHECK, "invalid lane index");
            k[q] |= uint32_t(lane) << (8 * b);
          }
        }
        Entry y = pop_t(V128), x = pop_t(V128);
        if (!live()) { push_cell(V128); break; }
        uint32_t idx = uint32_t(P.vconst.size() / 4);
        P.vconst.insert(P.vconst.end(), k, k + 4);
        uint32_t a = src(x), b = src(y);
        emit(OP_V_SHUFFLE, a, b, x.cell, 0, idx);
        push_cell(V128, last_emit);
        break;
      }
      case 0xFD15: case 0xFD16: case 0xFD18: case 0xFD19: case 0xFD1B: case 0xFD1D:
      case 0xFD1F: case 0xFD21: {  // extract_lane
        uint8_t lane = r.u8();
        static const std::map<uint16_t, std::pair<uint16_t, uint8_t>> m = {
            {0xFD15, {OP_V_EXTRACT8S, I32}}, {0xFD16, {OP_V_EXTRACT8U, I32}},
            {0xFD18, {OP_V_EXTRACT16S, I32}}, {0xFD19, {OP_V_EXTRACT16U, I32}},
            {0xFD1B, {OP_V_EXTRACT32, I32}}, {0xFD1D, {OP_V_EXTRACT64, I64}},
            {0xFD1F, {OP_V_EXTRACT32, F32}}, {0xFD21, {OP_V_EXTRACT64, F64}}};
        auto e = m.at(op);
        uint32_t lanes = e.first == OP_V_EXTRACT8S || e.first == OP_V_EXTRACT8U ? 16
                         : e.first == OP_V_EXTRACT16S || e.first == OP_V_EXTRACT16U ? 8
                         : e.first == OP_V_EXTRACT32 ? 4 : 2;
        if (lane >= lanes) fail(E_TYPECHECK, "invalid lane index");
        Entry v = pop_t(V128);
        if (!live()) { push_cell(e.second); break; }
        uint32_t a = src(v);
        emit(e.first, a, 0, v.cell, lane);
        push_cell(e.second, last_emit);
        break;
      }
      case 0xFD17: case 0xFD1A: case 0xFD1C: case 0xFD1E: case 0xFD20: case 0xFD22: {
        uint8_t lane = r.u8();
        static const std::map<uint16_t, std::pair<uint16_t, uint8_t>> m = {
            {0xFD17, {OP_V_REPLACE8, I32}}, {0xFD1A, {OP_V_REPLACE16, I32}},
            {0xFD1C, {OP_V_REPLACE32, I32}}, {0xFD1E, {OP_V_REPLACE64, I64}},
            {0xFD20, {OP_V_REPLACE32, F32}}, {0xFD22, {OP_V_REPLACE64, F64}}};
        auto e = m.at(op);
        uint32_t lanes = e.first == OP_V_REPLACE8 ? 16 : e.first == OP_V_REPLACE16 ? 8
                         : e.first == OP_V_REPLACE32 ? 4 : 2;
        if (lane >= lanes) fail(E_TYPECHECK, "invalid lane index");
        Entry s = pop_t(e.second), v = pop_t(V128);
        if (!live()) { push_cell(V128); break; }
        uint32_t a = src(v), b = src(s);
        emit(e.first, a, b, v.cell, lane);
        push_cell(V128, last_emit);
        break;
      }
      default: {
        char buf[96];
        snprintf(buf, sizeof buf, "opcode 0x%X not supported by the batched path", op);
        fail(E_UNSUPPORTED, buf);
      }
    }
  }
  if (r.p != r.end) fail(E_MALFORMED, "junk after function end");
  F.frame_cells = max_cell - frame_base;
  if (F.frame_cells > P.frame_cells) P.frame_cells = F.frame_cells;
}

// ------------------------------------------------------------------ module parsing
struct ConstVal {
  uint8_t type;
  uint32_t k[4];
};

// `ops`: the expression's instructions (its `end` included) join Program::init_ops --
// instantiation runs every constant expression through the interpreter loop, so each
// one is counted and priced (engine.cpp:13-17; instantiate/global.cpp:42, elem.cpp:25,39,
// data.cpp:27)
ConstVal eval_const(Reader &r, const Program &P, const std::vector<ConstVal> &globals,
                    std::vector<uint16_t> *ops) {
  ConstVal v{UNKNOWN, {0, 0, 0, 0}};
  for (;;) {
    uint8_t op = r.u8();
    ops->push_back(op == 0xFD ? 0xFD0C : op);
    if (op == 0x0B) break;
    switch (op) {
      case 0x41: v.type = I32; v.k[0] = uint32_t(int32_t(r.sleb(32))); break;
      case 0x42: { uint64_t x = uint64_t(r.sleb(64)); v.type = I64; v.k[0] = uint32_t(x); v.k[1] = uint32_t(x >> 32); break; }
      case 0x43: v.type = F32; for (int q = 0; q < 4; q++) v.k[0] |= uint32_t(r.u8()) << (8 * q); break;
      case 0x44: { uint64_t x = 0; for (int q = 0; q < 8; q++) x |= uint64_t(r.u8()) << (8 * q);
                   v.type = F64; v.k[0] = uint32_t(x); v.k[1] = uint32_t(x >> 32); break; }
      case 0xD0: v.type = r.u8(); v.k[0] = 0xFFFFFFFFu; break;
      case 0xD2: v.type = FUNCREF; v.k[0] = r.u32(); break;
      case 0x23: { uint32_t g = r.u32(); if (g >= globals.size()) throw Err{E_TYPECHECK, "unknown global"}; v = globals[g]; break; }
      case 0xFD: {
        if (r.u32() != 0x0C) throw Err{E_TYPECHECK, "constant expression required"};
        v.type = V128;
        for (int q = 0; q < 4; q++) for (int b = 0; b < 4; b++) v.k[q] |= uint32_t(r.u8()) << (8 * b);
        break;
      }
      default: throw Err{E_TYPECHECK, "constant expression required"};
    }
  }
  (void)P;
  return v;
}

// Peephole over the finished program: an i32 add (or ADD3) followed by an in-place
// xor-rotate of another cell with the sum (the add-xor-rotate step of BLAKE3's G, ChaCha's
// quarter round, ...) becomes one dispatch. The second instruction is removed and every
// pc reference is remapped; pairs whose second half is a branch/call target are kept.
static bool is_pc_branch(uint16_t op) {
  return op == OP_JMP || op == OP_BR_IF || op == OP_BR_UNLESS || op == OP_BR_IF_MOV1 ||
         op == OP_BR_IF_MOV2 || (op >= OP_BR_EQ && op <= OP_BR_GE_U_I);
}

// Short loops around every pc, for the kernel's scheduler (KParams::loops): every
// backward branch (pc -> t <= pc, br_table entries included) closes a loop [t, pc]; the
// innermost one around x is the shortest such span that contains x. Only innermost loops
// of fewer than kScanLoop instructions are kept: scan loops (`while (a[i] < p) i++`)
// whose data-dependent trip counts keep the other lanes waiting (see batch_kernel.hip).
constexpr uint32_t kScanLoop = 8;
void find_loops(Program &P) {
  const uint32_t n = uint32_t(P.code.size());
  std::vector<std::pair<uint32_t, uint32_t>> spans;
  for (uint32_t pc = 0; pc < n; pc++) {
    const DInstr &I = P.code[pc];
    const uint16_t op = I.w0 & 0x7FFF;
    if (is_pc_branch(op) && I.w3 <= pc) spans.push_back({I.w3, pc});
    if (op == OP_BR_TABLE) {
      const uint32_t labels = (I.w1 >> 16) & 0xFFFFu;   // B_: entries [imm, imm + B_]
      for (uint32_t k = 0; k <= labels && 2 * (I.w3 + k) < P.brtab.size(); k++)
        if (P.brtab[2 * (I.w3 + k)] <= pc) spans.push_back({P.brtab[2 * (I.w3 + k)], pc});
    }
  }
  P.loops.assign(2 * size_t(n) + 2, 0xFFFFFFFFu);
  std::vector<uint32_t> len(n + 1, 0xFFFFFFFFu);
  for (const auto &sp : spans)
    for (uint32_t x = sp.first; x <= sp.second; x++)
      if (sp.second - sp.first < len[x]) {
        len[x] = sp.second - sp.first;
        P.loops[2 * x] = sp.first;
        P.loops[2 * x + 1] = sp.second;
      }
  for (uint32_t x = 0; x < n; x++)
    if (len[x] != 0xFFFFFFFFu && len[x] + 1 >= kScanLoop) P.loops[2 * x] = P.loops[2 * x + 1] = 0xFFFFFFFFu;
}

void fuse_arx(Program &P) {
  const size_t n = P.code.size();
  std::vector<uint8_t> target(n + 1, 0);
  for (size_t pc = 0; pc < n; pc++) {
    const DInstr &I = P.code[pc];
    const uint16_t op = I.w0 & 0x7FFF;
    if ((is_pc_branch(op) || op == OP_CALL || op == OP_TAIL_CALL) && I.w3 < n) target[I.w3] = 1;
    if (op == OP_CALL || op == OP_CALL_INDIRECT) target[pc + 1] = 1;   // return pc
  }
  for (size_t k = 0; k + 1 < P.brtab.size(); k += 2)
    if (P.brtab[k] < n) target[P.brtab[k]] = 1;
  for (const auto &f : P.funcs)
    if (!f.imported) { target[f.entry_pc] = 1; target[f.body_pc] = 1; }
  std::vector<uint8_t> drop(n, 0);
  size_t fused = 0;
  for (size_t pc = 0; pc + 1 < n; pc++) {
    DInstr &I = P.code[pc], &J = P.code[pc + 1];
    const uint16_t op1 = I.w0 & 0x7FFF, op2 = J.w0 & 0x7FFF;
    if ((op1 != OP_I32_ADD && op1 != OP_I32_ADD3) || target[pc + 1] || drop[pc]) continue;
    if (op2 != OP_I32_XOR_ROTR_I && op2 != OP_I32_XOR_ROTL_I) continue;
    const uint32_t sum = I.w2 & 0xFFFF, ja = J.w1 & 0xFFFF, jb = J.w1 >> 16, jc = J.w2 & 0xFFFF;
    const uint32_t y = ja == sum ? jb : ja;
    if ((ja != sum && jb != sum) || jc != y || y == sum) continue;   // y = rot(y ^ sum)
    const uint32_t cnt = ((I.w0 >> 16) & 0xFF) + ((J.w0 >> 16) & 0xFF);
    if (cnt > 255 || y > 0xFFFF) continue;
    const uint32_t k = op2 == OP_I32_XOR_ROTR_I ? (J.w3 & 31u) : ((32u - (J.w3 & 31u)) & 31u);
    const uint32_t post = (J.w0 >> 24) & 0x7F;
    if (op1 == OP_I32_ADD) {
      I.w0 = OP_I32_ADD_XROTR_I | (cnt << 16) | (post << 24);
      I.w2 = sum | (y << 16);
      I.w3 = k;
    } else {
      I.w0 = OP_I32_ADD3_XROTR_I | (cnt << 16) | (post << 24);
      I.w3 = y | (k << 16);
    }
    if (cnt > P.max_wasm_instrs_per_dispatch) P.max_wasm_instrs_per_dispatch = cnt;
    P.dops[pc].insert(P.dops[pc].end(), P.dops[pc + 1].begin(), P.dops[pc + 1].end());
    drop[pc + 1] = 1;
    fused++;
  }
  if (!fused) return;
  std::vector<uint32_t> remap(n + 1);
  std::vector<DInstr> out;
  std::vector<std::vector<uint16_t>> dout;
  out.reserve(n - fused);
  for (size_t pc = 0; pc < n; pc++) {
    remap[pc] = uint32_t(out.size());
    if (!drop[pc]) { out.push_back(P.code[pc]); dout.push_back(std::move(P.dops[pc])); }
  }
  remap[n] = uint32_t(out.size());
  for (DInstr &I : out) {
    const uint16_t op = I.w0 & 0x7FFF;
    if ((is_pc_branch(op) || op == OP_CALL || op == OP_TAIL_CALL) && I.w3 <= n) I.w3 = remap[I.w3];
  }
  for (size_t k = 0; k + 1 < P.brtab.size(); k += 2)
    if (P.brtab[k] <= n) P.brtab[k] = remap[P.brtab[k]];
  for (auto &f : P.funcs)
    if (!f.imported) { f.entry_pc = remap[f.entry_pc]; f.body_pc = remap[f.body_pc]; }
  P.code.swap(out);
  P.dops.swap(dout);
}

// instantiate/import.cpp:35-42 isLimitMatched(provided, declared)
static bool limits_match(const HostImport &h, uint32_t min, bool has_max, uint32_t max) {
  if (h.min < min || (!h.has_max && has_max)) return false;
  if (h.has_max && has_max && h.max > max) return false;
  return true;
}

void parse_and_lower(const uint8_t *wasm, size_t len, Program &P,
                     const std::vector<HostImport> *imports) {
  if (len < 8 || memcmp(wasm, "\0asm\1\0\0\0", 8)) throw Err{0x23, "magic header not detected"};
  Reader r{wasm + 8, wasm + len};
  std::vector<uint32_t> decl_types;
  std::vector<ConstVal> gvals;
  uint32_t ncode = 0;
  while (r.p < r.end) {
    uint8_t sid = r.u8();
    uint32_t slen = r.u32();
    if (uint64_t(r.end - r.p) < slen) throw Err{E_MALFORMED, "section size mismatch"};
    Reader s{r.p, r.p + slen};
    switch (sid) {
      case 0: break;
      case 1: {
        uint32_t n = s.u32();
        for (uint32_t k = 0; k < n; k++) {
          if (s.u8() != 0x60) throw Err{E_MALFORMED, "malformed function type"};
          FuncType t;
          uint32_t np = s.u32();
          for (uint32_t q = 0; q < np; q++) t.params.push_back(s.u8());
          uint32_t nr = s.u32();
          for (uint32_t q = 0; q < nr; q++) t.results.push_back(s.u8());
          P.types.push_back(t);
        }
        break;
      }
      case 2: {
        uint32_t n = s.u32();
        for (uint32_t k = 0; k < n; k++) {
          std::string mod = s.name(), nm = s.name();
          uint8_t kind = s.u8();
          if (kind != 0) {
            // a table / memory / global import (instantiate/import.cpp:137-190)
            if (kind > 3) throw Err{E_MALFORMED, "malformed import kind"};
            uint8_t ty = 0, mut = 0, fl = 0;
            uint32_t mn = 0, mx = 0;
            if (kind == 1) ty = s.u8();
            if (kind == 1 || kind == 2) {
              fl = s.u8();
              mn = s.u32();
              if (fl & 1) mx = s.u32();
            } else {
              ty = s.u8();
              mut = s.u8();
            }
            const HostImport *h = nullptr;
            if (imports)
              for (const auto &x : *imports)
                if (x.module == mod && x.name == nm && x.kind == kind) { h = &x; break; }
            if (!h) throw Err{0x62, "unknown import " + mod + "." + nm};
            if (kind == 1) {
              if (h->type != ty || !limits_match(*h, mn, fl & 1, mx))
                throw Err{0x61, "incompatible import type " + mod + "." + nm};
              TableInfo t;
              t.type = h->type;
              t.min = h->min;
              t.has_max = h->has_max;
              t.max = h->max;
              P.tables.push_back(t);
              P.ntables = uint32_t(P.tables.size());
            } else if (kind == 2) {
              if (P.has_mem && !P.multi_memory) throw Err{0x51, "multiple memories"};
              if (!limits_match(*h, mn, fl & 1, mx))
                throw Err{0x61, "incompatible import type " + mod + "." + nm};
              if (h->min > 65536 || (h->has_max && h->max > 65536))
                throw Err{0x53, "memory size must be at most 65536 pages (4GiB)"};
              if (P.has_mem) {   // (a further memory: MultiMemories)
                if (P.xmems.size() >= kMaxXMem) throw Err{E_UNSUPPORTED, "more than 8 memories"};
                P.xmems.push_back(Program::MemLimits{h->min, h->has_max ? h->max : 65536u, h->has_max});
                continue;
              }
              P.has_mem = true;
              P.mem_min = h->min;
              P.mem_has_max = h->has_max;
              P.mem_max = h->has_max ? h->max : 65536;
            } else {
              if (h->type != ty || uint8_t(h->mut) != mut)
                throw Err{0x61, "incompatible import type " + mod + "." + nm};
              ConstVal v{ty, {h->value[0], h->value[1], h->value[2], h->value[3]}};
              gvals.push_back(v);
              P.global_types.push_back(ty);
              P.global_mut.push_back(mut);
            }
            continue;
          }
          FuncInfo f;
          f.type = s.u32();
          if (f.type >= P.types.size()) throw Err{E_TYPECHECK, "unknown type"};
          f.imported = true;
          f.import_module = mod;
          f.import_name = nm;
          P.funcs.push_back(f);
          P.n_imported++;
        }
        break;
      }
      case 3: {
        uint32_t n = s.u32();
        for (uint32_t k = 0; k < n; k++) {
          uint32_t t = s.u32();
          if (t >= P.types.size()) throw Err{E_TYPECHECK, "unknown type"};
          decl_types.push_back(t);
        }
        break;
      }
      case 4: {
        uint32_t n = s.u32();
        for (uint32_t k = 0; k < n; k++) {
          TableInfo t;
          t.type = s.u8();
          if (t.type != FUNCREF && t.type != EXTERNREF) throw Err{E_MALFORMED, "malformed reference type"};
          uint8_t fl = s.u8();
          t.min = s.u32();
          if (fl & 1) { t.has_max = true; t.max = s.u32(); }
          if (t.has_max && t.max < t.min) throw Err{0x43, "size minimum must not be greater than maximum"};
          P.tables.push_back(t);
        }
        P.ntables = uint32_t(P.tables.size());
        break;
      }
      case 5: {
        uint32_t n = s.u32();
        if (!P.multi_memory && (n > 1 || (n && P.has_mem))) throw Err{0x51, "multiple memories"};
        for (uint32_t k = 0; k < n; k++) {
          uint8_t fl = s.u8();
          Program::MemLimits ml;
          ml.min = s.u32();
          if (fl & 1) { ml.has_max = true; ml.max = s.u32(); }
          if (ml.min > 65536 || (ml.has_max && ml.max > 65536))
            throw Err{0x53, "memory size must be at most 65536 pages (4GiB)"};
          if (P.has_mem) {   // (a further memory: MultiMemories)
            if (P.xmems.size() >= kMaxXMem) throw Err{E_UNSUPPORTED, "more than 8 memories"};
            P.xmems.push_back(ml);
            continue;
          }
          P.has_mem = true;
          P.mem_min = ml.min;
          P.mem_has_max = ml.has_max;
          if (ml.has_max) P.mem_max = ml.max;
        }
        break;
      }
      case 6: {
        uint32_t n = s.u32();
        for (uint32_t k = 0; k < n; k++) {
          uint8_t t = s.u8();
          uint8_t mut = s.u8();
          ConstVal v = eval_const(s, P, gvals, &P.init_ops);
          if (v.type != t) throw Err{E_TYPECHECK, "type mismatch in global init"};
          gvals.push_back(v);
          P.global_types.push_back(t);
          P.global_mut.push_back(mut);
        }
        break;
      }
      case 7: {
        uint32_t n = s.u32();
        for (uint32_t k = 0; k < n; k++) {
          std::string nm = s.name();
          uint8_t kind = s.u8();
          uint32_t idx = s.u32();
          if (kind == 0) P.exports.push_back(ExportFunc{nm, idx});
          if (kind == 1) P.table_exports.push_back(ExportFunc{nm, idx});
          if (kind == 3) P.global_exports.push_back(ExportFunc{nm, idx});
        }
        break;
      }
      case 8: P.start_func = s.u32(); break;
      case 9: {
        uint32_t n = s.u32();
        for (uint32_t k = 0; k < n; k++) {
          // elem.cpp / binary format: bit 0 passive-or-declarative, bit 1 explicit
          // table (active) or declarative (passive), bit 2 items as const expressions
          uint32_t flags = s.u32();
          if (flags > 7) throw Err{E_MALFORMED, "malformed elements segment kind"};
          ElemSeg e;
          e.active = !(flags & 1);
          e.declarative = (flags & 3) == 3;
          if (e.active) {
            if (flags & 2) e.table = s.u32();
            ConstVal off = eval_const(s, P, gvals, &P.init_ops);
            e.offset = off.k[0];
          }
          if (flags & 3) {
            uint8_t k = s.u8();   // elemkind 0x00 (= funcref) or a reftype
            e.type = (flags & 4) ? k : FUNCREF;
          }
          uint32_t m = s.u32();
          for (uint32_t q = 0; q < m; q++) {
            if (flags & 4) {
              e.items.push_back(eval_const(s, P, gvals, &P.init_ops).k[0]);
            } else {   // a function index: the loader makes it `ref.func i; end` (segment.cpp:152-161)
              e.items.push_back(s.u32());
              P.init_ops.push_back(0xD2);
              P.init_ops.push_back(0x0B);
            }
          }
          P.elems.push_back(e);
        }
        break;
      }
      case 10: {
        ncode = s.u32();
        if (ncode != decl_types.size())
          throw Err{0x29, "function and code section have inconsistent lengths"};
        for (uint32_t k = 0; k < ncode; k++) {
          uint32_t blen = s.u32();
          const uint8_t *bend = s.p + blen;
          FuncInfo f;
          f.type = decl_types[k];
          uint32_t ng = s.u32();
          uint64_t total = 0;
          for (uint32_t g = 0; g < ng; g++) {
            uint32_t c = s.u32();
            uint8_t t = s.u8();
            total += c;
            if (total > 50000) throw Err{0x30, "too many locals"};
            f.local_types.insert(f.local_types.end(), c, t);
          }
          f.code_off = uint32_t(s.p - wasm);
          f.code_len = uint32_t(bend - s.p);
          s.p = bend;
          P.funcs.push_back(f);
        }
        break;
      }
      case 11: {
        uint32_t n = s.u32();
        for (uint32_t k = 0; k < n; k++) {
          uint32_t flags = s.u32();
          DataSeg d;
          d.active = !(flags & 1);
          if (flags == 2) d.mem = s.u32();   // (segment.cpp:316-323)
          if (d.active) d.offset = eval_const(s, P, gvals, &P.init_ops).k[0];
          uint32_t m = s.u32();
          if (uint64_t(s.end - s.p) < m) throw Err{E_MALFORMED, "length out of bounds"};
          d.bytes.assign(s.p, s.p + m);
          s.p += m;
          P.datas.push_back(d);
        }
        break;
      }
      case 12: s.u32(); break;
      default: throw Err{0x25, "malformed section id"};
    }
    r.p += slen;
  }
  if (decl_types.size() != ncode) throw Err{0x29, "function and code section have inconsistent lengths"};
  // canonical structural type ids (call_indirect compares FunctionTypes by value)
  for (size_t k = 0; k < P.types.size(); k++) {
    uint32_t id = uint32_t(k);
    for (size_t q = 0; q < k; q++)
      if (P.types[q] == P.types[k]) { id = P.type_canon[q]; break; }
    P.type_canon.push_back(id);
  }
  // globals -> cells [0, G)
  uint32_t gc = 0;
  for (size_t k = 0; k < gvals.size(); k++) {
    P.global_cell.push_back(gc);
    uint32_t w = cells_of(gvals[k].type);
    for (uint32_t q = 0; q < w; q++) P.global_init.push_back(gvals[k].k[q]);
    gc += w;
  }
  P.global_cells = gc;
  // tables at instantiation (instantiate/table.cpp + elem.cpp): `min` null refs, then
  // the active element segments in order
  for (auto &e : P.elems) {
    if (e.active && e.table >= P.ntables) throw Err{E_TYPECHECK, "unknown table"};
    if (e.active && e.type != P.tables[e.table].type) throw Err{E_TYPECHECK, "type mismatch"};
  }
  std::vector<std::vector<uint32_t>> timg(P.ntables);
  for (uint32_t t = 0; t < P.ntables; t++) timg[t].assign(P.tables[t].min, 0xFFFFFFFFu);
  for (auto &e : P.elems) {
    if (!e.active) continue;
    auto &T = timg[e.table];
    if (uint64_t(e.offset) + e.items.size() > T.size())
      throw Err{0x64, "elements segment does not fit"};
    for (size_t q = 0; q < e.items.size(); q++) T[e.offset + q] = e.items[q];
  }
  if (P.ntables) P.table0 = timg[0];
  // several tables, an externref table or an exported table (the host may write it,
  // WasmEdge_BatchTableSetData): per-lane tables from the start
  P.mut_tables = P.ntables > 1 || (P.ntables && P.tables[0].type != FUNCREF) ||
                 !P.table_exports.empty();
  for (auto &e : P.table_exports)
    if (e.func >= P.ntables) throw Err{E_TYPECHECK, "unknown table"};
  for (auto &e : P.global_exports)
    if (e.func >= P.global_types.size()) throw Err{E_TYPECHECK, "unknown global"};
  for (auto &d : P.datas) {
    if (!d.active) continue;
    const uint32_t nm = (P.has_mem ? 1u : 0u) + uint32_t(P.xmems.size());
    if (d.mem >= nm) throw Err{uint8_t(P.multi_memory && nm ? 0x47 : E_TYPECHECK), "unknown memory"};
    const uint32_t mn = d.mem ? P.xmems[d.mem - 1].min : P.mem_min;
    if (uint64_t(d.offset) + d.bytes.size() > uint64_t(mn) * 65536)
      throw Err{0x63, "data segment does not fit"};
  }
  if (P.start_func >= 0) {   // validator.cpp: the start function has type [] -> []
    if (uint64_t(P.start_func) >= P.funcs.size()) throw Err{E_TYPECHECK, "unknown function"};
    const FuncType &st = P.types[P.funcs[P.start_func].type];
    if (!st.params.empty() || !st.results.empty()) throw Err{E_TYPECHECK, "invalid start function"};
  }
  // lower
  const Program before = P;
  VarInfo vi;
  vi.locals.resize(P.funcs.size());
  {
    // per-instance entry points: exported functions (the host passes per-instance
    // arguments) and functions reachable through a table (call_indirect from anywhere)
    std::vector<uint8_t> entry(P.funcs.size(), 0);
    for (const auto &e : P.exports) if (e.func < entry.size()) entry[e.func] = 1;
    for (const auto &e : P.elems) for (uint32_t f : e.items) if (f < entry.size()) entry[f] = 1;
    for (uint32_t f = P.n_imported; f < P.funcs.size(); f++) {
      const FuncInfo &F = P.funcs[f];
      const size_t np = P.types[F.type].params.size();
      vi.locals[f].assign(np + F.local_types.size(), 0);
      if (entry[f]) std::fill(vi.locals[f].begin(), vi.locals[f].begin() + np, 1);
    }
  }
  for (int round = 0;; round++) {
    try {
      vi.changed = false;
      Lowerer L(P, wasm, vi);
      std::vector<CallFix> callfix;
      for (uint32_t f = P.n_imported; f < P.funcs.size(); f++) L.lower_function(f, callfix);
      // a call to a function lowered after its caller learns the callee's body pc and
      // local cells (the locals the call zeroes: helper.cpp:155-161) only now
      for (auto &c : callfix) {
        DInstr &I = P.code[c.instr];
        // (the c field is 16 bits, as emit() checks for cell indices)
        if (P.funcs[c.callee].local_cells > 0xFFFFu)
          throw Err{E_UNSUPPORTED, "callee locals exceed the DBC encoding (65535 cells)"};
        I.w3 = P.funcs[c.callee].body_pc;
        I.w2 = (I.w2 & 0xFFFF0000u) | P.funcs[c.callee].local_cells;
      }
      if (!vi.changed || round >= 16) {
        if (vi.changed) P.divergent_mem = true;   // not settled: assume divergence
        break;
      }
      const bool mt = P.mut_tables;
      P = before;
      P.mut_tables = mt;
    } catch (NeedMutTables &) {
      P = before;
      P.mut_tables = true;
    }
  }
  if (P.mut_tables) {
    // per-lane table words: each table starts with min + kTableGrowLimit slots (bounded by
    // its max; a grow past them widens the tables at run time); element segment pool for table.init; active and declarative segments
    // start dropped (elem.cpp)
    P.init_edropped.assign((P.elems.size() + 31) / 32 + (P.elems.empty() ? 1 : 0), 0u);
    for (uint32_t t = 0; t < P.ntables; t++) {
      const TableInfo &T = P.tables[t];
      uint64_t cap = uint64_t(T.min) + kTableGrowLimit;
      if (T.has_max && cap > T.max) cap = T.max;
      if (cap > 0xFFFFFFFFull) cap = 0xFFFFFFFFull;
      if (uint64_t(P.tab_words) + cap > (1u << 24)) throw Err{E_UNSUPPORTED, "tables too large"};
      P.tabinfo.push_back(P.tab_words);
      P.tabinfo.push_back(uint32_t(cap));
      P.tab_image.insert(P.tab_image.end(), timg[t].begin(), timg[t].end());
      P.tab_image.resize(P.tab_words + cap, 0xFFFFFFFFu);
      P.tab_words += uint32_t(cap);
    }
    for (size_t k = 0; k < P.elems.size(); k++) {
      const ElemSeg &e = P.elems[k];
      P.elem_off.push_back(uint32_t(P.elem_pool.size()));
      P.elem_len.push_back(uint32_t(e.items.size()));
      P.elem_pool.insert(P.elem_pool.end(), e.items.begin(), e.items.end());
      if (e.active || e.declarative) P.init_edropped[k >> 5] |= 1u << (k & 31);
    }
  }
  fuse_arx(P);
  find_loops(P);
  // every instruction's opcode list holds exactly the `cnt` instructions it retires
  if (P.dops.size() != P.code.size()) throw Err{E_UNSUPPORTED, "internal: opcode lists out of step"};
  for (size_t pc = 0; pc < P.code.size(); pc++)
    if (((P.code[pc].w0 >> 16) & 0xFFu) != P.dops[pc].size())
      throw Err{E_UNSUPPORTED, "internal: opcode list of pc " + std::to_string(pc) + " does not match its count"};
  if (P.code.size() >= DBC_MAX_PC) throw Err{E_UNSUPPORTED, "module too large for 20-bit pcs"};
}

}  // namespace

uint64_t build_cost_pool(const Program &P, const uint64_t *tab, uint64_t limit,
                         std::vector<uint32_t> &off, std::vector<uint64_t> &pool, bool *exceeded) {
  off.assign(P.code.size() + 1, 0);
  pool.clear();
  for (size_t pc = 0; pc < P.code.size(); pc++) {
    off[pc] = uint32_t(pool.size());
    uint64_t s = 0;
    for (uint16_t op : P.dops[pc]) { s += tab[op]; pool.push_back(s); }
  }
  off[P.code.size()] = uint32_t(pool.size());
  if (pool.empty()) pool.push_back(0);
  uint64_t c = 0;
  *exceeded = false;
  for (uint16_t op : P.init_ops) {
    const uint64_t n = c + tab[op];
    if (n > limit) { *exceeded = true; break; }
    c = n;
  }
  return c;
}

std::string load_program(const uint8_t *wasm, size_t len, Program &out, uint8_t *errcode,
                         bool exact_globals, const std::vector<HostImport> *imports, bool tail_call,
                         bool multi_memory) {
  try {
    out = Program();
    out.exact_globals = exact_globals;
    out.tail_call = tail_call;
    out.multi_memory = multi_memory;
    parse_and_lower(wasm, len, out, imports);
    *errcode = 0;
    return "";
  } catch (const Err &e) {
    *errcode = e.code;
    return e.msg;
  }
}

int find_export(const Program &p, const std::string &name) {
  for (auto &e : p.exports)
    if (e.name == name) return int(e.func);
  return -1;
}

const char *dop_name(uint16_t op) {
  static const char *names[] = {
#define DBC_NAME(n) #n,
      DBC_OPS(DBC_NAME)
#undef DBC_NAME
  };
  return op < OP_DBC_NUM_OPS ? names[op] : "?";
}

}  // namespace wb
