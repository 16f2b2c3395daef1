// dbc_ops.h -- per-lane operation helpers shared by the gfx950 kernel and the host-side
// test emulator (emu.cpp). Semantics restated from the reference with file:line.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

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

// ------------------------------------------------------------- linear memory access
// m points at word 0 of this lane (stride 64 words between consecutive words).
WB_HD uint32_t mword(const uint32_t *m, uint32_t w) {
  return m[(size_t)w << WB_MSHIFT];
}
WB_HD uint64_t mload(const uint32_t *m, uint32_t ea, uint32_t n) {
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
WB_HD uint64_t mload_aligned(const uint32_t *m, uint32_t ea, uint32_t n) {
  const uint32_t w = ea >> 2;
  const uint32_t x = mword(m, w);
  if (n == 8) return (uint64_t)x | ((uint64_t)mword(m, w + 1) << 32);
  if (n == 4) return x;
  const uint32_t y = x >> ((ea & 3u) * 8u);
  return n == 1 ? (y & 0xFFu) : (y & 0xFFFFu);
}
WB_HD void mstore_aligned(uint32_t *m, uint32_t ea, uint32_t n, uint64_t v) {
  uint32_t *p = &m[(size_t)(ea >> 2) << WB_MSHIFT];
  if (n >= 4) {
    p[0] = (uint32_t)v;
    if (n == 8) p[(size_t)1 << WB_MSHIFT] = (uint32_t)(v >> 32);
  } else if (n == 2) {
    reinterpret_cast<uint16_t *>(p)[(ea & 3u) >> 1] = (uint16_t)v;
  } else {
    reinterpret_cast<uint8_t *>(p)[ea & 3u] = (uint8_t)v;
  }
}
WB_HD void mstore(uint32_t *m, uint32_t ea, uint32_t n, uint64_t v) {
  if ((ea & 3u) == 0 && n >= 4) {
    m[(size_t)(ea >> 2) << WB_MSHIFT] = (uint32_t)v;
    if (n == 8) m[(size_t)((ea >> 2) + 1) << WB_MSHIFT] = (uint32_t)(v >> 32);
    return;
  }
  for (uint32_t k = 0; k < n; k++) {
    const uint32_t a = ea + k;
    reinterpret_cast<uint8_t *>(&m[(size_t)(a >> 2) << WB_MSHIFT])[a & 3u] = (uint8_t)(v >> (8 * k));
  }
}
WB_HD uint8_t mbyte(const uint32_t *m, uint32_t a) {
  return reinterpret_cast<const uint8_t *>(&m[(size_t)(a >> 2) << WB_MSHIFT])[a & 3u];
}
WB_HD void mbyte_set(uint32_t *m, uint32_t a, uint8_t v) {
  reinterpret_cast<uint8_t *>(&m[(size_t)(a >> 2) << WB_MSHIFT])[a & 3u] = v;
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
