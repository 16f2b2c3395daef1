// dbc_ops.h -- per-lane operation helpers shared by the gfx950 kernel and the host-side
// test emulator (emu.cpp). Semantics restated from the reference with file:line.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>
#include "dbc.h"

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define WB_HD __host__ __device__ __forceinline__
#else
#define WB_HD static inline
#endif
// operand fields of the current DInstr (w1/w2/w3 are in scope in the dispatch loop)
#define A_ (w1 & 0xFFFFu)
#define B_ (w1 >> 16)
#define C_ (w2 & 0xFFFFu)
#define D_ (w2 >> 16)
#define IMM w3

#ifndef WB_MSHIFT
#define WB_MSHIFT 6   /* words of one lane are 64 words apart (lane-interleaved) */
#endif

namespace wbops {

WB_HD float f32(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
WB_HD uint32_t b32(float f) { uint32_t b; memcpy(&b, &f, 4); return b; }
WB_HD double f64(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
WB_HD uint64_t b64(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }

// x86-64 SSE NaN selection (what the reference's g++ build produces):
// a NaN result takes the first NaN operand, quieted; an invalid operation with no NaN
// operand gives the default NaN with the sign bit set.
// Mask selects: the interpreter's fast loop must not branch per lane, and clang lowers
// some nested `?:` on per-lane conditions to divergent branches; these never do.
WB_HD uint32_t sel32(bool c, uint32_t x, uint32_t y) {
  const uint32_t m = 0u - (uint32_t)c;
  return (m & x) | (~m & y);
}
WB_HD uint64_t sel64(bool c, uint64_t x, uint64_t y) {
  const uint64_t m = 0ull - (uint64_t)c;
  return (m & x) | (~m & y);
}
WB_HD uint32_t nan_fix32(uint32_t r, uint32_t a, uint32_t b) {
  const bool rn = (r & 0x7FFFFFFFu) > 0x7F800000u;
  const bool an = (a & 0x7FFFFFFFu) > 0x7F800000u;
  const bool bn = (b & 0x7FFFFFFFu) > 0x7F800000u;
  return sel32(rn, sel32(an, a | 0x00400000u, sel32(bn, b | 0x00400000u, 0xFFC00000u)), r);
}
WB_HD uint64_t nan_fix64(uint64_t r, uint64_t a, uint64_t b) {
  const uint64_t ab = 0x7FFFFFFFFFFFFFFFull, inf = 0x7FF0000000000000ull, q = 0x0008000000000000ull;
  const bool rn = (r & ab) > inf, an = (a & ab) > inf, bn = (b & ab) > inf;
  return sel64(rn, sel64(an, a | q, sel64(bn, b | q, 0xFFF8000000000000ull)), r);
}
WB_HD bool isnan32(uint32_t a) { return (a & 0x7FFFFFFFu) > 0x7F800000u; }
WB_HD bool isnan64(uint64_t a) {
  return (a & 0x7FFFFFFFFFFFFFFFull) > 0x7FF0000000000000ull;
}
// ceil/floor/trunc (unary_numeric.ipp:73-86, 358-398): g++ -O2 expands std::ceil/floor/trunc
// inline with SSE2 (|x| >= 2^23 or unordered -> x), so a NaN operand comes back unchanged,
// signalling ones included (tools/nan_probe.cpp); nearest calls libm roundeven, which quiets.
WB_HD uint32_t nan_keep32(uint32_t r, uint32_t a) { return sel32(isnan32(a), a, r); }
WB_HD uint64_t nan_keep64(uint64_t r, uint64_t a) { return sel64(isnan64(a), a, r); }

// Gas metering (statistics.h:79-91 addCost): the sum Old + Cost (wrapping in 64 bits) past
// the limit fails without being added. `pool[j]` = the cost of a DBC's first j+1
// instructions (KParams::cost_pool). gas_step prices instructions [from, to) in order; on
// CostLimitExceeded it sets `add` to the count through the failing instruction.
WB_HD uint64_t gas_at(const uint64_t *pool, uint32_t j) { return j ? pool[j] - pool[j - 1] : pool[0]; }
WB_HD bool gas_step(const uint64_t *pool, uint32_t from, uint32_t to, uint64_t limit,
                    uint64_t &cost, int32_t &add) {
  for (uint32_t j = from; j < to; j++) {
    const uint64_t nc = cost + gas_at(pool, j);
    if (nc > limit) { add = (int32_t)(j + 1); return true; }
    cost = nc;
  }
  return false;
}
// After the main op: the instructions after it, then a taken branch's count correction --
// tcnt = -k: its landing DBC re-prices its first k instructions (the landing list's prefix
// is returned here); tcnt = +1: an if-false jump into an else arm also retires the `else`
// (controlInstr.cpp:23-28).
WB_HD bool gas_tail(const uint64_t *pool, uint32_t from, uint32_t cnt, int32_t jtc,
                    const uint64_t *landing, uint64_t c_else, uint64_t limit, uint64_t &cost,
                    int32_t &add) {
  if (gas_step(pool, from, cnt, limit, cost, add)) return true;
  if (jtc < 0) cost -= landing[(uint32_t)(-jtc) - 1u];
  for (int32_t q = 0; q < jtc; q++) {
    const uint64_t nc = cost + c_else;
    if (nc > limit) { add = (int32_t)cnt + q + 1; return true; }
    cost = nc;
  }
  return false;
}

// binary_numeric.ipp:155-191 (scalar min/max with its NaN/zero rules; raw NaN payload)
WB_HD uint32_t fmin32(uint32_t a, uint32_t b) {
  const bool zz = ((a | b) & 0x7FFFFFFFu) == 0 && a != b;
  const uint32_t lt = sel32(f32(b) < f32(a), b, a);
  return sel32(isnan32(b), b, sel32(zz, 0x80000000u, sel32(isnan32(a), a, lt)));
}
WB_HD uint32_t fmax32(uint32_t a, uint32_t b) {
  const bool zz = ((a | b) & 0x7FFFFFFFu) == 0 && a != b;
  const uint32_t gt = sel32(f32(a) < f32(b), b, a);
  return sel32(isnan32(b), b, sel32(zz, 0u, sel32(isnan32(a), a, gt)));
}
WB_HD uint64_t fmin64(uint64_t a, uint64_t b) {
  const bool zz = ((a | b) & 0x7FFFFFFFFFFFFFFFull) == 0 && a != b;
  const uint64_t lt = sel64(f64(b) < f64(a), b, a);
  return sel64(isnan64(b), b, sel64(zz, 0x8000000000000000ull, sel64(isnan64(a), a, lt)));
}
WB_HD uint64_t fmax64(uint64_t a, uint64_t b) {
  const bool zz = ((a | b) & 0x7FFFFFFFFFFFFFFFull) == 0 && a != b;
  const uint64_t gt = sel64(f64(a) < f64(b), b, a);
  return sel64(isnan64(b), b, sel64(zz, 0ull, sel64(isnan64(a), a, gt)));
}
// binary_numeric.ipp:442-475 (vector fmin/fmax lanes)
WB_HD uint32_t vfmin32(uint32_t x, uint32_t y) {
  uint32_t r = x | y;
  if (f32(x) < f32(y)) r = x;
  if (f32(x) > f32(y)) r = y;
  if (isnan32(x)) r = x;
  if (isnan32(y)) r = y;
  return r;
}
WB_HD uint32_t vfmax32(uint32_t x, uint32_t y) {
  uint32_t r = x & y;
  if (f32(x) < f32(y)) r = y;
  if (f32(x) > f32(y)) r = x;
  if (isnan32(x)) r = x;
  if (isnan32(y)) r = y;
  return r;
}
WB_HD uint64_t vfmin64(uint64_t x, uint64_t y) {
  uint64_t r = x | y;
  if (f64(x) < f64(y)) r = x;
  if (f64(x) > f64(y)) r = y;
  if (isnan64(x)) r = x;
  if (isnan64(y)) r = y;
  return r;
}
WB_HD uint64_t vfmax64(uint64_t x, uint64_t y) {
  uint64_t r = x & y;
  if (f64(x) < f64(y)) r = y;
  if (f64(x) > f64(y)) r = x;
  if (isnan64(x)) r = x;
  if (isnan64(y)) r = y;
  return r;
}

// cast_numeric.ipp:39-82: trunc with traps. Returns 0 or an ErrCode (branch-free).
// in32: input is f32; sgn: signed target; out64: 64-bit target.
WB_HD uint32_t trunc_chk(double z, bool in32, bool sgn, bool out64, uint64_t &res) {
  const double t = trunc(z);
  double mn, mx;
  if (out64) {
    mn = sgn ? -9223372036854775808.0 : 0.0;
    mx = sgn ? 9223372036854775808.0 : 18446744073709551616.0;   // (TIn)max rounds up
  } else {
    mn = sgn ? -2147483648.0 : 0.0;
    mx = sgn ? (in32 ? 2147483648.0 : 2147483647.0) : (in32 ? 4294967296.0 : 4294967295.0);
  }
  const bool better = !in32 && !out64;   // sizeof(TIn) > sizeof(TOut): f64 -> i32
  const bool oor = better ? (t < mn || t > mx) : (t < mn || t >= mx);
  const uint32_t e = sel32(z != z, 0x86u, sel32(__builtin_isinf(z) || oor, 0x85u, 0u));
  const double tc = e ? 0.0 : t;
  if (out64) res = sgn ? (uint64_t)(int64_t)tc : (uint64_t)tc;
  else res = sgn ? (uint64_t)(uint32_t)(int32_t)tc : (uint64_t)(uint32_t)tc;
  return e;
}
// cast_numeric.ipp:84-123 (saturating)
WB_HD uint64_t trunc_sat(double z, bool in32, bool sgn, bool out64) {
  const uint64_t lo = out64 ? (sgn ? 0x8000000000000000ull : 0) : (sgn ? 0x80000000ull : 0);
  const uint64_t hi = out64 ? (sgn ? 0x7FFFFFFFFFFFFFFFull : ~0ull) : (sgn ? 0x7FFFFFFFull : 0xFFFFFFFFull);
  uint64_t r;
  const uint32_t e = trunc_chk(z, in32, sgn, out64, r);
  return sel64(z != z, 0, sel64(e == 0, r, sel64(z < 0, lo, hi)));
}

// ------------------------------------------------------------- SIMD128 lane-wise ops
// The v128 value is four 32-bit cells, little-endian: lane k of width W bytes is bits
// [8*W*k, 8*W*(k+1)) of the 128-bit value. All loops below have constant trip counts and
// are unrolled, so lane indices fold to constants (no scratch).
WB_HD uint32_t vlane(const uint32_t *v, uint32_t W, uint32_t k) {
  const uint32_t bit = 8 * W * k;
  return W == 4 ? v[k] : (v[bit >> 5] >> (bit & 31)) & ((1u << (8 * W)) - 1u);
}
WB_HD void vlane_set(uint32_t *v, uint32_t W, uint32_t k, uint32_t x) {
  const uint32_t bit = 8 * W * k;
  if (W == 4) { v[k] = x; return; }
  const uint32_t m = ((1u << (8 * W)) - 1u) << (bit & 31);
  v[bit >> 5] = (v[bit >> 5] & ~m) | ((x << (bit & 31)) & m);
}
WB_HD int32_t vsx(uint32_t x, uint32_t W) {   // sign-extend a W-byte lane
  return W == 4 ? (int32_t)x : (int32_t)(x << (32 - 8 * W)) >> (32 - 8 * W);
}
WB_HD int32_t vclamp(int32_t x, int32_t lo, int32_t hi) { return x < lo ? lo : x > hi ? hi : x; }

// OP_V_BINX: c = op(a, b) for the binary 0xFD ops without a dedicated DOp
// (binary_numeric.ipp:203-567: compares 264-313 (V1 < V2 etc. on signed/unsigned lanes),
// narrow 285-314, add/sub_sat 349-398, min/max 412-440, avgr 477-491, extmul 493-552,
// q15mulr 554-566; i32x4.dot engine.cpp:1579-1593).
WB_HD void vbinx(uint32_t sub, const uint32_t *x, const uint32_t *y, uint32_t *r) {
  uint32_t o[4] = {0, 0, 0, 0};
#define WB_LW(W, EXPR) { _Pragma("unroll") for (uint32_t k = 0; k < 16 / (W); k++) { \
    const uint32_t a = vlane(x, W, k), b = vlane(y, W, k); \
    const int32_t as = vsx(a, W), bs = vsx(b, W); (void)a; (void)b; (void)as; (void)bs; \
    vlane_set(o, W, k, (uint32_t)(EXPR)); } } break
  switch (sub) {
    // i8x16 / i16x8 ordered compares: lt_s lt_u gt_s gt_u le_s le_u ge_s ge_u
    case 0x25: WB_LW(1, as < bs ? ~0u : 0u);  case 0x26: WB_LW(1, a < b ? ~0u : 0u);
    case 0x27: WB_LW(1, as > bs ? ~0u : 0u);  case 0x28: WB_LW(1, a > b ? ~0u : 0u);
    case 0x29: WB_LW(1, as <= bs ? ~0u : 0u); case 0x2A: WB_LW(1, a <= b ? ~0u : 0u);
    case 0x2B: WB_LW(1, as >= bs ? ~0u : 0u); case 0x2C: WB_LW(1, a >= b ? ~0u : 0u);
    case 0x2F: WB_LW(2, as < bs ? ~0u : 0u);  case 0x30: WB_LW(2, a < b ? ~0u : 0u);
    case 0x31: WB_LW(2, as > bs ? ~0u : 0u);  case 0x32: WB_LW(2, a > b ? ~0u : 0u);
    case 0x33: WB_LW(2, as <= bs ? ~0u : 0u); case 0x34: WB_LW(2, a <= b ? ~0u : 0u);
    case 0x35: WB_LW(2, as >= bs ? ~0u : 0u); case 0x36: WB_LW(2, a >= b ? ~0u : 0u);
    // saturating add/sub, min/max, rounding average
    case 0x6F: WB_LW(1, vclamp(as + bs, -128, 127));
    case 0x70: WB_LW(1, a + b > 255u ? 255u : a + b);
    case 0x72: WB_LW(1, vclamp(as - bs, -128, 127));
    case 0x73: WB_LW(1, a > b ? a - b : 0u);
    case 0x76: WB_LW(1, as > bs ? b : a);  case 0x77: WB_LW(1, a > b ? b : a);
    case 0x78: WB_LW(1, bs > as ? b : a);  case 0x79: WB_LW(1, b > a ? b : a);
    case 0x7B: WB_LW(1, (a + b + 1) >> 1);
    case 0x82: WB_LW(2, vclamp((as * bs + 0x4000) >> 15, -32768, 32767));
    case 0x8F: WB_LW(2, vclamp(as + bs, -32768, 32767));
    case 0x90: WB_LW(2, a + b > 65535u ? 65535u : a + b);
    case 0x92: WB_LW(2, vclamp(as - bs, -32768, 32767));
    case 0x93: WB_LW(2, a > b ? a - b : 0u);
    case 0x96: WB_LW(2, as > bs ? b : a);  case 0x97: WB_LW(2, a > b ? b : a);
    case 0x98: WB_LW(2, bs > as ? b : a);  case 0x99: WB_LW(2, b > a ? b : a);
    case 0x9B: WB_LW(2, (a + b + 1) >> 1);
    case 0xB6: WB_LW(4, as > bs ? b : a);  case 0xB7: WB_LW(4, a > b ? b : a);
    case 0xB8: WB_LW(4, bs > as ? b : a);  case 0xB9: WB_LW(4, b > a ? b : a);
    // narrow: x's lanes then y's, saturated to the half width
    case 0x65: case 0x66: case 0x85: case 0x86: {
      const uint32_t W = (sub == 0x65 || sub == 0x66) ? 1 : 2, n = 8 / W;
      const bool sg = sub == 0x65 || sub == 0x85;
      const int32_t lo = sg ? -(1 << (8 * W - 1)) : 0;
      const int32_t hi = sg ? (1 << (8 * W - 1)) - 1 : (1 << (8 * W)) - 1;
      _Pragma("unroll") for (uint32_t k = 0; k < 8; k++) {
        if (k < n) {
          vlane_set(o, W, k, (uint32_t)vclamp(vsx(vlane(x, 2 * W, k), 2 * W), lo, hi));
          vlane_set(o, W, k + n, (uint32_t)vclamp(vsx(vlane(y, 2 * W, k), 2 * W), lo, hi));
        }
      }
      break;
    }
    // extmul low/high (s, u) into 16- and 32-bit lanes
    case 0x9C: case 0x9D: case 0x9E: case 0x9F: case 0xBC: case 0xBD: case 0xBE: case 0xBF: {
      const uint32_t W = sub < 0xBC ? 1 : 2, n = 8 / W, off = (sub & 1) ? n : 0;
      const bool sg = (sub & 2) == 0;
      _Pragma("unroll") for (uint32_t k = 0; k < 8; k++) {
        if (k < n) {
          const uint32_t a = vlane(x, W, k + off), b = vlane(y, W, k + off);
          const uint32_t p = sg ? (uint32_t)(vsx(a, W) * vsx(b, W)) : a * b;
          vlane_set(o, 2 * W, k, p);
        }
      }
      break;
    }
    case 0xDC: case 0xDD: case 0xDE: case 0xDF: {   // i64x2.extmul_{low,high}_i32x4_{s,u}
      const uint32_t off = (sub & 1) ? 2 : 0;
      _Pragma("unroll") for (uint32_t k = 0; k < 2; k++) {
        const uint64_t p = (sub & 2) ? (uint64_t)x[k + off] * y[k + off]
                                     : (uint64_t)((int64_t)(int32_t)x[k + off] * (int32_t)y[k + off]);
        o[2 * k] = (uint32_t)p; o[2 * k + 1] = (uint32_t)(p >> 32);
      }
      break;
    }
    case 0xBA: {   // i32x4.dot_i16x8_s: pairwise products summed (wrapping)
      _Pragma("unroll") for (uint32_t k = 0; k < 4; k++)
        o[k] = (uint32_t)(vsx(vlane(x, 2, 2 * k), 2) * vsx(vlane(y, 2, 2 * k), 2)) +
               (uint32_t)(vsx(vlane(x, 2, 2 * k + 1), 2) * vsx(vlane(y, 2, 2 * k + 1), 2));
      break;
    }
    default: break;
  }
#undef WB_LW
  r[0] = o[0]; r[1] = o[1]; r[2] = o[2]; r[3] = o[3];
}

WB_HD uint32_t demote_bits(uint64_t a) {   // cast_numeric.ipp f32.demote_f64 (x86 NaN)
  uint32_t r = b32((float)f64(a));
  if (isnan64(a)) r = (uint32_t)(a >> 32 & 0x80000000u) | 0x7FC00000u | (uint32_t)((a >> 29) & 0x003FFFFFu);
  return r;
}
WB_HD uint64_t promote_bits(uint32_t a) {
  uint64_t r = b64((double)f32(a));
  if (isnan32(a)) r = ((uint64_t)(a & 0x80000000u) << 32) | 0x7FF8000000000000ull | ((uint64_t)(a & 0x003FFFFFu) << 29);
  return r;
}

// OP_V_UNX: c = op(a) for the unary 0xFD ops without a dedicated DOp
// (unary_numeric.ipp:98-415: extend 121-165, extadd_pairwise 167-178, abs/neg 180-207,
// popcnt 209-216, trunc_sat 230-267, convert 269-282, demote/promote 284-297,
// ceil/floor/trunc/nearest 372-412).
WB_HD void vunx(uint32_t sub, const uint32_t *x, uint32_t *r) {
  uint32_t o[4] = {0, 0, 0, 0};
#define WB_LU(W, EXPR) { _Pragma("unroll") for (uint32_t k = 0; k < 16 / (W); k++) { \
    const uint32_t a = vlane(x, W, k); const int32_t as = vsx(a, W); (void)a; (void)as; \
    vlane_set(o, W, k, (uint32_t)(EXPR)); } } break
  switch (sub) {
    case 0x60: WB_LU(1, as < 0 ? 0u - a : a);
    case 0x61: WB_LU(1, 0u - a);
    case 0x62: WB_LU(1, __builtin_popcount(a));
    case 0x80: WB_LU(2, as < 0 ? 0u - a : a);
    case 0x81: WB_LU(2, 0u - a);
    case 0x67: WB_LU(4, nan_keep32(b32(ceilf(f32(a))), a));
    case 0x68: WB_LU(4, nan_keep32(b32(floorf(f32(a))), a));
    case 0x69: WB_LU(4, nan_keep32(b32(truncf(f32(a))), a));
    case 0x6A: WB_LU(4, nan_fix32(b32(rintf(f32(a))), a, a));
    case 0xF8: WB_LU(4, (uint32_t)trunc_sat((double)f32(a), true, true, false));
    case 0xF9: WB_LU(4, (uint32_t)trunc_sat((double)f32(a), true, false, false));
    case 0xFA: WB_LU(4, b32((float)(int32_t)a));
    case 0xFB: WB_LU(4, b32((float)a));
    case 0x74: case 0x75: case 0x7A: case 0x94: {
      _Pragma("unroll") for (uint32_t k = 0; k < 2; k++) {
        const uint64_t a = x[2 * k] | ((uint64_t)x[2 * k + 1] << 32);
        const double d = f64(a);
        const double t = sub == 0x74 ? ceil(d) : sub == 0x75 ? floor(d) : sub == 0x7A ? trunc(d) : rint(d);
        const uint64_t v = sub == 0x94 ? nan_fix64(b64(t), a, a) : nan_keep64(b64(t), a);
        o[2 * k] = (uint32_t)v; o[2 * k + 1] = (uint32_t)(v >> 32);
      }
      break;
    }
    case 0x7C: case 0x7D: case 0x7E: case 0x7F: {   // extadd_pairwise
      const uint32_t W = sub <= 0x7D ? 1 : 2;
      const bool sg = (sub & 1) == 0;
      _Pragma("unroll") for (uint32_t k = 0; k < 8; k++) {
        if (k < 8 / W) {
          const uint32_t a = vlane(x, W, 2 * k), b = vlane(x, W, 2 * k + 1);
          vlane_set(o, 2 * W, k, sg ? (uint32_t)(vsx(a, W) + vsx(b, W)) : a + b);
        }
      }
      break;
    }
    case 0x87: case 0x88: case 0x89: case 0x8A: case 0xA7: case 0xA8: case 0xA9: case 0xAA: {
      const uint32_t W = sub <= 0x8A ? 1 : 2, n = 8 / W, off = (sub & 1) ? 0 : n;
      const bool sg = sub == 0x87 || sub == 0x88 || sub == 0xA7 || sub == 0xA8;
      _Pragma("unroll") for (uint32_t k = 0; k < 8; k++) {
        if (k < n) {
          const uint32_t a = vlane(x, W, k + off);
          vlane_set(o, 2 * W, k, sg ? (uint32_t)vsx(a, W) : a);
        }
      }
      break;
    }
    case 0xC7: case 0xC8: case 0xC9: case 0xCA: {   // i64x2.extend_{low,high}_i32x4_{s,u}
      const uint32_t off = (sub & 1) ? 0 : 2;
      const bool sg = sub <= 0xC8;
      _Pragma("unroll") for (uint32_t k = 0; k < 2; k++) {
        o[2 * k] = x[k + off];
        o[2 * k + 1] = sg && (int32_t)x[k + off] < 0 ? ~0u : 0u;
      }
      break;
    }
    case 0xFC: case 0xFD: {   // i32x4.trunc_sat_f64x2_{s,u}_zero
      _Pragma("unroll") for (uint32_t k = 0; k < 2; k++)
        o[k] = (uint32_t)trunc_sat(f64(x[2 * k] | ((uint64_t)x[2 * k + 1] << 32)), false, sub == 0xFC, false);
      break;
    }
    case 0xFE: case 0xFF: {   // f64x2.convert_low_i32x4_{s,u}
      _Pragma("unroll") for (uint32_t k = 0; k < 2; k++) {
        const uint64_t v = b64(sub == 0xFE ? (double)(int32_t)x[k] : (double)x[k]);
        o[2 * k] = (uint32_t)v; o[2 * k + 1] = (uint32_t)(v >> 32);
      }
      break;
    }
    case 0x5E:   // f32x4.demote_f64x2_zero
      o[0] = demote_bits(x[0] | ((uint64_t)x[1] << 32));
      o[1] = demote_bits(x[2] | ((uint64_t)x[3] << 32));
      break;
    case 0x5F: {   // f64x2.promote_low_f32x4
      const uint64_t p0 = promote_bits(x[0]), p1 = promote_bits(x[1]);
      o[0] = (uint32_t)p0; o[1] = (uint32_t)(p0 >> 32); o[2] = (uint32_t)p1; o[3] = (uint32_t)(p1 >> 32);
      break;
    }
    default: break;
  }
#undef WB_LU
  r[0] = o[0]; r[1] = o[1]; r[2] = o[2]; r[3] = o[3];
}

// ------------------------------------------------------------- linear memory access
// A lane's linear memory as seen by the step code. The emulator passes a plain pointer
// (its memory is contiguous per instance, WB_MSHIFT 0). The kernel passes a GMem: the
// wave's 64 memories interleaved in granules of 2^g words -- word w of lane l at
// ((w >> g) * 64 + l) * 2^g + (w & (2^g - 1)) words from the wave's base (g = 0: word
// interleave; the kernel's `p` already includes the lane's l * 2^g).
struct GMem {
  uint32_t *p;
  uint32_t g;
};
WB_HD uint32_t *mw(uint32_t *m, uint32_t w) { return &m[(size_t)w << WB_MSHIFT]; }
WB_HD const uint32_t *mw(const uint32_t *m, uint32_t w) { return &m[(size_t)w << WB_MSHIFT]; }
WB_HD size_t goff(uint32_t w, uint32_t g) {
  return ((size_t)(w >> g) << (6 + g)) | (size_t)(w & ((1u << g) - 1u));
}
WB_HD uint32_t *mw(GMem m, uint32_t w) { return &m.p[goff(w, m.g)]; }
// The paged view (the kernel's per-lane step): words below `rwords` (the reserved pages)
// as GMem; word w of page q = w >> 14 beyond them in the wave's pool row pt[q - rpages],
// the same 64-lane interleave within the row (`loff` = the lane's l * 2^g). Only accesses
// the caller bounds-checked against the lane's pages come here, and every page below that
// has a row.
struct GMemP {
  uint32_t *p;
  uint32_t g;
  uint32_t rwords;
  const uint64_t *pt;
  uint32_t loff;
};
WB_HD uint32_t *mw(GMemP m, uint32_t w) {
  if (w < m.rwords) return &m.p[goff(w, m.g)];
  uint32_t *row = (uint32_t *)(uintptr_t)m.pt[(w - m.rwords) >> 14];
  return &row[m.loff + goff(w & 16383u, m.g)];
}

template <class M> WB_HD uint32_t mword(M m, uint32_t w) { return *mw(m, w); }
template <class M> WB_HD uint64_t mload(M m, uint32_t ea, uint32_t n) {
  const uint32_t w = ea >> 2, s = (ea & 3u) * 8u;
  if (s == 0) {
    if (n == 4) return mword(m, w);
    if (n == 8) return (uint64_t)mword(m, w) | ((uint64_t)mword(m, w + 1) << 32);
    const uint32_t x = mword(m, w);
    return n == 1 ? (x & 0xFFu) : (x & 0xFFFFu);
  }
  const uint32_t last = (ea + n - 1) >> 2;
  const uint64_t x0 = mword(m, w);
  const uint64_t x1 = last > w ? mword(m, w + 1) : 0;
  const uint64_t x2 = last > w + 1 ? mword(m, w + 2) : 0;
  const uint64_t lo = x0 | (x1 << 32);
  const uint64_t r = (lo >> s) | (x2 << (64 - s));
  return n == 8 ? r : (r & ((1ull << (n * 8)) - 1));
}
// Naturally aligned accesses (ea % min(n,4) == 0), branch-free per lane: n is uniform,
// an access never straddles a 32-bit word except the two words of an 8-byte one.
template <class M> WB_HD uint64_t mload_aligned(M m, uint32_t ea, uint32_t n) {
  const uint32_t w = ea >> 2;
  const uint32_t x = mword(m, w);
  if (n == 8) return (uint64_t)x | ((uint64_t)mword(m, w + 1) << 32);
  if (n == 4) return x;
  const uint32_t y = x >> ((ea & 3u) * 8u);
  return n == 1 ? (y & 0xFFu) : (y & 0xFFFFu);
}
template <class M> WB_HD void mstore_aligned(M m, uint32_t ea, uint32_t n, uint64_t v) {
  uint32_t *p = mw(m, ea >> 2);
  if (n >= 4) {
    p[0] = (uint32_t)v;
    if (n == 8) *mw(m, (ea >> 2) + 1) = (uint32_t)(v >> 32);
  } else if (n == 2) {
    reinterpret_cast<uint16_t *>(p)[(ea & 3u) >> 1] = (uint16_t)v;
  } else {
    reinterpret_cast<uint8_t *>(p)[ea & 3u] = (uint8_t)v;
  }
}
template <class M> WB_HD void mstore(M m, uint32_t ea, uint32_t n, uint64_t v) {
  if ((ea & 3u) == 0 && n >= 4) {
    *mw(m, ea >> 2) = (uint32_t)v;
    if (n == 8) *mw(m, (ea >> 2) + 1) = (uint32_t)(v >> 32);
    return;
  }
  for (uint32_t k = 0; k < n; k++) {
    const uint32_t a = ea + k;
    reinterpret_cast<uint8_t *>(mw(m, a >> 2))[a & 3u] = (uint8_t)(v >> (8 * k));
  }
}
template <class M> WB_HD uint8_t mbyte(M m, uint32_t a) {
  return reinterpret_cast<const uint8_t *>(mw(m, a >> 2))[a & 3u];
}
template <class M> WB_HD void mbyte_set(M m, uint32_t a, uint8_t v) {
  reinterpret_cast<uint8_t *>(mw(m, a >> 2))[a & 3u] = v;
}

// A memory-0 load op as XLD carries it (memories past the first): bytes read, sign
// extension, a 64-bit cell pair, a v128 result (memory.ipp:12-38, 70-220)
struct LdShape { uint32_t n; bool sx, w64, v; };
WB_HD __attribute__((always_inline)) LdShape ld_shape(uint32_t op) {
  switch (op) {
    case OP_LD8S32: return {1, true, false, false};
    case OP_LD8U32: return {1, false, false, false};
    case OP_LD16S32: return {2, true, false, false};
    case OP_LD16U32: return {2, false, false, false};
    case OP_LD32: return {4, false, false, false};
    case OP_LD8S64: return {1, true, true, false};
    case OP_LD8U64: return {1, false, true, false};
    case OP_LD16S64: return {2, true, true, false};
    case OP_LD16U64: return {2, false, true, false};
    case OP_LD32S64: return {4, true, true, false};
    case OP_LD32U64: return {4, false, true, false};
    case OP_LD64: return {8, false, true, false};
    case OP_LD128: return {16, false, false, true};
    case OP_V_LD8SPLAT: return {1, false, false, true};
    case OP_V_LD16SPLAT: return {2, false, false, true};
    case OP_V_LD32SPLAT: case OP_V_LD32ZERO: return {4, false, false, true};
    default: return {8, false, false, true};   // the 64-bit extending, splat and zero forms
  }
}
// the v128 a load form makes of its bytes (x: the first 8, hi: bytes 8..15 of LD128)
WB_HD __attribute__((always_inline)) void v128_of_load(uint32_t op, uint64_t x, uint64_t hi, uint32_t o[4]) {
  o[0] = o[1] = o[2] = o[3] = 0;
  switch (op) {
    case OP_LD128:
      o[0] = (uint32_t)x; o[1] = (uint32_t)(x >> 32); o[2] = (uint32_t)hi; o[3] = (uint32_t)(hi >> 32);
      break;
    case OP_V_LD8X8S: case OP_V_LD8X8U:
      for (int k = 0; k < 4; k++) {
        uint32_t b0 = (x >> (16 * k)) & 0xFF, b1 = (x >> (16 * k + 8)) & 0xFF;
        if (op == OP_V_LD8X8S) { b0 = (uint32_t)(int32_t)(int8_t)b0 & 0xFFFF; b1 = (uint32_t)(int32_t)(int8_t)b1 & 0xFFFF; }
        o[k] = b0 | (b1 << 16);
      }
      break;
    case OP_V_LD16X4S: case OP_V_LD16X4U:
      for (int k = 0; k < 4; k++) {
        const uint32_t h = (x >> (16 * k)) & 0xFFFF;
        o[k] = op == OP_V_LD16X4S ? (uint32_t)(int32_t)(int16_t)h : h;
      }
      break;
    case OP_V_LD32X2S: case OP_V_LD32X2U:
      for (int k = 0; k < 2; k++) {
        const uint32_t v = (uint32_t)(x >> (32 * k));
        o[2 * k] = v;
        o[2 * k + 1] = op == OP_V_LD32X2S ? (((int32_t)v < 0) ? 0xFFFFFFFFu : 0u) : 0u;
      }
      break;
    case OP_V_LD8SPLAT: o[0] = o[1] = o[2] = o[3] = ((uint32_t)x & 0xFF) * 0x01010101u; break;
    case OP_V_LD16SPLAT: { const uint32_t h = (uint32_t)x & 0xFFFF; o[0] = o[1] = o[2] = o[3] = h | (h << 16); break; }
    case OP_V_LD32SPLAT: o[0] = o[1] = o[2] = o[3] = (uint32_t)x; break;
    case OP_V_LD64SPLAT: o[0] = o[2] = (uint32_t)x; o[1] = o[3] = (uint32_t)(x >> 32); break;
    case OP_V_LD32ZERO: o[0] = (uint32_t)x; break;
    default: o[0] = (uint32_t)x; o[1] = (uint32_t)(x >> 32); break;   // LD64ZERO
  }
}

WB_HD uint32_t clz32(uint32_t x) { return x ? __builtin_clz(x) : 32; }
WB_HD uint32_t ctz32(uint32_t x) { return x ? __builtin_ctz(x) : 32; }
WB_HD uint64_t clz64(uint64_t x) { return x ? __builtin_clzll(x) : 64; }
WB_HD uint64_t ctz64(uint64_t x) { return x ? __builtin_ctzll(x) : 64; }
WB_HD uint32_t rotl32(uint32_t x, uint32_t k) { k &= 31; return k ? (x << k) | (x >> (32 - k)) : x; }
WB_HD uint32_t rotr32(uint32_t x, uint32_t k) { k &= 31; return k ? (x >> k) | (x << (32 - k)) : x; }
WB_HD uint64_t rotl64(uint64_t x, uint64_t k) { k &= 63; return k ? (x << k) | (x >> (64 - k)) : x; }
WB_HD uint64_t rotr64(uint64_t x, uint64_t k) { k &= 63; return k ? (x >> k) | (x << (64 - k)) : x; }

}  // namespace
namespace wbops {
WB_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33; return k;
}
}  // namespace wbops
using namespace wbops;
