// nan_probe.cpp -- what g++ -O2 (x86-64, SSE2 baseline, the reference's default build)
// does with NaN operands for the expression SHAPES of the reference's numeric templates.
// Own code, not the reference's: each function restates one shape
// (include/executor/engine/{binary,unary,cast}_numeric.ipp) so the NaN payload rules the
// oracle and the device follow are pinned to the compiler's actual code.
//   g++ -O2 -std=c++17 -o /tmp/nan_probe tools/nan_probe.cpp && /tmp/nan_probe
// Expected (g++ 11.4, glibc 2.35): add/mul keep the FIRST (lhs) NaN operand, quieted;
// ceil/floor/trunc return a NaN unchanged (inline SSE2 expansion, no libm call); nearest,
// sqrt, demote and promote quiet it.
#include <cmath>
#include <cstdint>
#include <cstdio>
union V { float f; double d; uint32_t u[4]; uint64_t q[2];
          float vf __attribute__((vector_size(16))); double vd __attribute__((vector_size(16))); };
__attribute__((noinline)) void add_(V &a, const V &b) { a.f += b.f; }          // binary_numeric.ipp:16
__attribute__((noinline)) void mul_(V &a, const V &b) { a.f *= b.f; }          // :32
__attribute__((noinline)) void addd_(V &a, const V &b) { a.d += b.d; }
__attribute__((noinline)) void vadd_(V &a, const V &b) { a.vf += b.vf; }       // vector add
__attribute__((noinline)) void ceil_(V &v) { v.f = std::ceil(v.f); }          // unary_numeric.ipp:74
__attribute__((noinline)) void floord_(V &v) { v.d = std::floor(v.d); }       // :79
__attribute__((noinline)) void vceil_(V &v) {                                  // :358-372
  using VT [[gnu::vector_size(16)]] = float;
  VT &R = v.vf;
  R = VT{std::ceil(R[0]), std::ceil(R[1]), std::ceil(R[2]), std::ceil(R[3])};
}
__attribute__((noinline)) void near_(V &v) { v.f = __builtin_roundevenf(v.f); } // roundeven.h:45
__attribute__((noinline)) void sqrt_(V &v) { v.f = std::sqrt(v.f); }           // :94
__attribute__((noinline)) void demote_(V &v) { v.f = static_cast<float>(v.d); } // cast_numeric.ipp
int main() {
  V a, b;
  a.u[0] = 0x7FA00002; b.u[0] = 0x7FC00001; add_(a, b); printf("f32 sNaN+qNaN   %08x\n", a.u[0]);
  a.u[0] = 0x7FC00001; b.u[0] = 0x7FA00002; add_(a, b); printf("f32 qNaN+sNaN   %08x\n", a.u[0]);
  a.u[0] = 0xFFC00000; b.u[0] = 0x7FC00001; mul_(a, b); printf("f32 -NaN*qNaN   %08x\n", a.u[0]);
  a.q[0] = 0x7FF4000000000001ull; b.q[0] = 0x7FF8000000000123ull; addd_(a, b);
  printf("f64 sNaN+qNaN   %016llx\n", (unsigned long long)a.q[0]);
  a.u[0] = 0x7FA00002; b.u[0] = 0x7FC00001; a.u[1] = b.u[1] = 0; vadd_(a, b);
  printf("f32x4 sNaN+qNaN %08x\n", a.u[0]);
  a.u[0] = 0xFFA00002; ceil_(a); printf("ceil sNaN       %08x\n", a.u[0]);
  a.q[0] = 0x7FF4000000000001ull; floord_(a); printf("floor f64 sNaN  %016llx\n", (unsigned long long)a.q[0]);
  a.u[0] = 0xFFA00002; a.u[1] = 0x7FA00001; vceil_(a); printf("f32x4 ceil sNaN %08x %08x\n", a.u[0], a.u[1]);
  a.u[0] = 0xFFA00002; near_(a); printf("nearest sNaN    %08x\n", a.u[0]);
  a.u[0] = 0xFFA00002; sqrt_(a); printf("sqrt sNaN       %08x\n", a.u[0]);
  a.u[0] = 0xBF800000; sqrt_(a); printf("sqrt -1         %08x\n", a.u[0]);
  a.q[0] = 0x7FF4000000000123ull; demote_(a); printf("demote sNaN     %08x\n", a.u[0]);
  return 0;
}
