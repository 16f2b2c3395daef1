// Frame-in-VGPR building blocks on gfx950 (one wave alone; s_memtime deltas over
// 64-fold .rept blocks): an operand round trip through LDS versus GPR-index mode
// (s_set_gpr_idx_on / v_mov / s_set_gpr_idx_off). Tuning aid only.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define REP "64"
#define CL "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", \
           "v138", "v139", "v140", "v40", "v41", "v42", "s20", "s21", "s22"
__global__ void __launch_bounds__(64) kbench(uint64_t *out, uint32_t *chk) {
  __shared__ uint32_t lds[4096];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  uint64_t t0, t1;
  int k = 0;
  const uint32_t a = threadIdx.x * 4;
#define T(body, ...) \
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)); \
  asm volatile("s_mov_b32 s20, 5\n s_mov_b32 s21, 7\n s_mov_b32 s22, 9\n v_mov_b32 v133, 1\n v_mov_b32 v135, 2\n" \
               ".rept " REP "\n" body "\n.endr\n" __VA_ARGS__); \
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)); \
  if (threadIdx.x == 0) out[k] = t1 - t0; k++;
  T("", ::: CL)
  // 1: LDS round trip: write result, read it back as the next operand, add
  T("ds_write_b32 %0, v40\n ds_read_b32 v41, %0\n s_waitcnt lgkmcnt(0)\n v_add_u32 v40, v41, 1", :: "v"(a) : CL)
  // 2: LDS two-operand dispatch body: 2 reads, add, write (reads depend on the last write)
  T("ds_read_b32 v41, %0\n ds_read_b32 v42, %0 offset:256\n s_waitcnt lgkmcnt(0)\n v_add_u32 v40, v41, v42\n ds_write_b32 %0, v40", :: "v"(a) : CL)
  // 3: gpr-index two-operand body: v[128+s20] + v[128+s21] -> v[128+s22]... -> chained via s20
  T("s_set_gpr_idx_on s20, gpr_idx(SRC0)\n v_mov_b32 v41, v128\n s_set_gpr_idx_idx s21\n v_mov_b32 v42, v128\n s_set_gpr_idx_off\n"
    " v_add_u32 v40, v41, v42\n s_set_gpr_idx_on s20, gpr_idx(DST)\n v_mov_b32 v128, v40\n s_set_gpr_idx_off", ::: CL)
  // 4: same with s_nop 0 after each index change
  T("s_set_gpr_idx_on s20, gpr_idx(SRC0)\n s_nop 0\n v_mov_b32 v41, v128\n s_set_gpr_idx_idx s21\n s_nop 0\n v_mov_b32 v42, v128\n s_set_gpr_idx_off\n"
    " v_add_u32 v40, v41, v42\n s_set_gpr_idx_on s20, gpr_idx(DST)\n s_nop 0\n v_mov_b32 v128, v40\n s_set_gpr_idx_off", ::: CL)
  // 5: just on/off pairs
  T("s_set_gpr_idx_on s20, gpr_idx(SRC0)\n s_set_gpr_idx_off", ::: CL)
  // 6: v_add dependent (reference)
  T("v_add_u32 v40, v40, 1", ::: CL)
  // 7: s_load_dwordx8 + wait (instruction fetch of the next TInstr)
  T("s_load_dwordx8 s[24:31], %0, 0x0\n s_waitcnt lgkmcnt(0)", :: "s"(out) : CL, "s24","s25","s26","s27","s28","s29","s30","s31")
  // 8: getpc+add+addc+setpc (the dispatch jump)
  T("s_getpc_b64 s[24:25]\n s_add_u32 s24, s24, 12\n s_addc_u32 s25, s25, 0\n s_setpc_b64 s[24:25]\n", ::: CL, "s24", "s25")
  // 9: one-operand body through gpr index (mov32-like): read a, write c
  T("s_set_gpr_idx_on s20, gpr_idx(SRC0)\n v_mov_b32 v41, v128\n s_set_gpr_idx_mode gpr_idx(DST)\n s_set_gpr_idx_idx s20\n v_mov_b32 v128, v41\n s_set_gpr_idx_off", ::: CL)
  // 10: SRC0 index with the add reading an indexed operand directly: v40 = v[128+i] + v42
  T("s_set_gpr_idx_on s20, gpr_idx(SRC0)\n v_add_u32 v40, v128, v40\n s_set_gpr_idx_off", ::: CL)
  // 11: 4 independent v_add
  T("v_add_u32 v40, v40, 1\n v_add_u32 v41, v41, 1\n v_add_u32 v42, v42, 1\n v_add_u32 v130, v130, 1", ::: CL)
  // 12: 4 independent s_add
  T("s_add_u32 s20, s20, 1\n s_add_u32 s21, s21, 1\n s_add_u32 s22, s22, 1\n s_add_u32 s24, s24, 1", ::: CL, "s24")
  // 13: 4 dependent s_add
  T("s_add_u32 s20, s20, 1\n s_add_u32 s20, s20, 1\n s_add_u32 s20, s20, 1\n s_add_u32 s20, s20, 1", ::: CL)
  // 14: 4x s_set_gpr_idx_idx
  T("s_set_gpr_idx_idx s20\n s_set_gpr_idx_idx s21\n s_set_gpr_idx_idx s22\n s_set_gpr_idx_idx s20", ::: CL)
  // 15: mixed: 2 s_add indep + 2 v_add indep interleaved
  T("s_add_u32 s20, s20, 1\n v_add_u32 v40, v40, 1\n s_add_u32 s21, s21, 1\n v_add_u32 v41, v41, 1", ::: CL)
  // 16: s_setpc to next with precomputed target (s_add+s_addc+setpc)
  T("s_getpc_b64 s[24:25]\n s_add_u32 s24, s24, 12\n s_addc_u32 s25, s25, 0\n s_setpc_b64 s[24:25]\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0", ::: CL, "s24", "s25")
  // correctness: v[128+5] after chains (lane values)
  uint32_t r0, r1;
  asm volatile("s_mov_b32 s20, 5\n v_mov_b32 v133, 11\n v_mov_b32 v135, 31\n s_mov_b32 s21, 7\n"
               "s_set_gpr_idx_on s20, gpr_idx(SRC0)\n v_mov_b32 %0, v128\n s_set_gpr_idx_idx s21\n v_mov_b32 %1, v128\n s_set_gpr_idx_off\n"
               : "=v"(r0), "=v"(r1) :: CL);
  uint32_t r2;
  asm volatile("s_mov_b32 s20, 6\n v_mov_b32 v40, 77\n s_set_gpr_idx_on s20, gpr_idx(DST)\n v_mov_b32 v128, v40\n s_set_gpr_idx_off\n v_mov_b32 %0, v134"
               : "=v"(r2) :: CL);
  if (threadIdx.x == 0) { chk[0] = r0; chk[1] = r1; chk[2] = r2; }
}

int main() {
  uint64_t *out; uint32_t *chk;
  hipMalloc(&out, 64 * 8); hipMemset(out, 0, 64 * 8);
  hipMalloc(&chk, 64); hipMemset(chk, 0, 64);
  const char *names[] = {"empty", "LDS round trip + add", "LDS 2-op body (2 reads, add, write)",
    "gpr-idx 2-op body", "gpr-idx 2-op body + nops", "idx on/off", "v_add dep", "s_load_x8+wait",
    "getpc+add+addc+setpc", "gpr-idx mov32 body", "gpr-idx add with indexed src0",
    "4 v_add indep", "4 s_add indep", "4 s_add dep", "4 s_set_gpr_idx_idx", "2 s_add+2 v_add indep",
    "getpc+add+addc+setpc+4 nops"};
  for (int it = 0; it < 3; it++) {
    hipLaunchKernelGGL(kbench, dim3(1), dim3(64), 0, 0, out, chk);
    hipDeviceSynchronize();
  }
  uint64_t h[64]; uint32_t c[4];
  hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
  hipMemcpy(c, chk, sizeof c, hipMemcpyDeviceToHost);
  for (int i = 0; i < 17; i++)
    printf("%2d %-40s %8.2f ticks/rep\n", i, names[i], (double)(h[i] - h[0]) / 64.0);
  printf("check: v[128+5]=%u (want 11) v[128+7]=%u (want 31) v134=%u (want 77)\n", c[0], c[1], c[2]);
  int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeClockRate, 0);
  printf("device clock attr %d kHz (s_memtime ticks at 100 MHz)\n", rate);
  return 0;
}
