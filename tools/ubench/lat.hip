// Latency / issue-cost microbenchmarks for the interpreter's dispatch building blocks
// (one wave alone on a CU, s_memtime deltas over 64-fold .rept blocks). Tuning aid only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP "64"
__global__ void kbench(const uint32_t *buf, uint64_t *out) {
  __shared__ uint32_t lds[1024];
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  uint64_t t0, t1;
  int k = 0;
#define T(body, ...) \
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0)); \
  asm volatile(".rept " REP "\n" body "\n.endr" __VA_ARGS__); \
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1)); \
  if (threadIdx.x == 0) out[k] = t1 - t0; k++;
  // 0: empty
  T("")
  // 1: s_load_dwordx4 + wait (scalar-cache hit latency)
  T("s_load_dwordx4 s[20:23], %0, 0x0\n s_waitcnt lgkmcnt(0)", :: "s"(buf) : "s20","s21","s22","s23")
  // 2: ds_read_b32 + wait
  T("ds_read_b32 v40, %0\n s_waitcnt lgkmcnt(0)", :: "v"(threadIdx.x * 4) : "v40")
  // 3: ds_read_b128 uniform address (broadcast) + wait
  T("ds_read_b128 v[40:43], %0\n s_waitcnt lgkmcnt(0)", :: "v"(0) : "v40","v41","v42","v43")
  // 4: s_load + ds_read both outstanding, one wait
  T("s_load_dwordx4 s[20:23], %0, 0x0\n ds_read_b32 v40, %1\n s_waitcnt lgkmcnt(0)", :: "s"(buf), "v"(threadIdx.x*4) : "s20","s21","s22","s23","v40")
  // 5: dependent SALU add
  T("s_add_u32 s20, s20, 1", ::: "s20")
  // 6: independent SALU
  T("s_add_u32 s20, s21, 1\n s_add_u32 s22, s23, 1", ::: "s20","s22")
  // 7: VALU add dependent
  T("v_add_u32 v40, v40, 1", ::: "v40")
  // 8: s_branch to next instruction (taken)
  T("s_branch 1f\n s_nop 0\n1:", ::: )
  // 9: s_cmp + s_cbranch_scc1 not taken
  T("s_cmp_eq_u32 s20, 12345\n s_cbranch_scc1 2f\n2:", ::: "s20")
  // 10: s_getpc + s_add + s_setpc to next
  T("s_getpc_b64 s[20:21]\n s_add_u32 s20, s20, 12\n s_addc_u32 s21, s21, 0\n s_setpc_b64 s[20:21]\n", ::: "s20","s21")
  // 11: v_readfirstlane -> s_add dependent
  T("v_readfirstlane_b32 s20, v41\n s_add_u32 s21, s20, 1", ::: "s20","s21")
  // 12: global_load_dwordx4 uniform + wait (L1/L2 hit)
  T("global_load_dwordx4 v[40:43], %0, off\n s_waitcnt vmcnt(0)", :: "v"(buf) : "v40","v41","v42","v43")
  // 13: s_buffer? s_load_dword dependent chain: address from previous load (pointer chase)
  T("s_load_dwordx2 s[20:21], %0, 0x0\n s_waitcnt lgkmcnt(0)\n s_load_dwordx2 s[22:23], %0, 0x0\n s_waitcnt lgkmcnt(0)", :: "s"(buf) : "s20","s21","s22","s23")
  // 14: ds_read_b32 -> v_add -> ds_write_b32 chain (an interpreter dispatch body)
  T("ds_read_b32 v40, %0\n ds_read_b32 v41, %0 offset:256\n s_waitcnt lgkmcnt(0)\n v_add_u32 v40, v40, v41\n ds_write_b32 %0, v40 offset:512", :: "v"(threadIdx.x*4) : "v40","v41")
  // 15: v_add_u32 v, s, v  (address formation) + ds_read + wait
  T("v_add_u32 v40, s0, %0\n ds_read_b32 v41, v40\n s_waitcnt lgkmcnt(0)", :: "v"(threadIdx.x*4) : "v40","v41")
  // 16: s_and/s_lshr decode pair
  T("s_and_b32 s20, s21, 0xffff\n s_lshr_b32 s22, s21, 16", ::: "s20","s22")
  // 17: s_mov_b64 x2
  T("s_mov_b64 s[20:21], s[22:23]\n s_mov_b64 s[24:25], s[26:27]", ::: "s20","s21","s24","s25")
  // 18: s_cmp + s_cbranch_scc1 taken to next
  T("s_cmp_eq_u32 s20, s20\n s_cbranch_scc1 3f\n s_nop 0\n3:", ::: )
  // 19: ds_write_b32 only
  T("ds_write_b32 %0, v41", :: "v"(threadIdx.x*4) : )
  // 20: s_load_dwordx8 + wait
  T("s_load_dwordx8 s[20:27], %0, 0x0\n s_waitcnt lgkmcnt(0)", :: "s"(buf) : "s20","s21","s22","s23","s24","s25","s26","s27")
  // 21: v_readfirstlane x4 then s_and on the last
  T("v_readfirstlane_b32 s20, v40\n v_readfirstlane_b32 s21, v41\n v_readfirstlane_b32 s22, v42\n v_readfirstlane_b32 s23, v43\n s_and_b32 s24, s20, s23", ::: "s20","s21","s22","s23","s24")
  // 22: v_cmp -> s_and exec -> s_cbranch_scc0 not taken (a compiled branch's lane test)
  T("v_cmp_le_i32_e32 vcc, 2, v41\n s_and_b64 s[20:21], vcc, exec\n s_cbranch_scc0 4f\n4:", ::: "s20","s21","vcc")
  // 23: readfirstlane + nop + v_cmp_ne + s_and + cbranch (the return record's uniformity test)
  T("v_readfirstlane_b32 s20, v40\n s_nop 1\n v_cmp_ne_u32_e64 s[22:23], s20, v40\n s_and_b64 s[22:23], s[22:23], exec\n s_cbranch_scc1 5f\n5:", ::: "s20","s22","s23")
  // 24: 12 independent SALU (issue rate of a transfer's scalar checks)
  T("s_add_u32 s20, s20, 4\n s_cmp_ge_u32 s20, s21\n s_cmp_le_u32 s22, s23\n s_cselect_b32 s24, s23, s24\n s_cmp_ge_u32 s22, s24\n s_add_u32 s25, s22, 0x20\n s_cmp_ge_u32 s25, s24\n s_mov_b32 s26, 0x60\n s_mov_b32 s27, 0x60\n s_mov_b32 s28, 0x60\n s_mov_b32 s29, 0x60\n s_mov_b32 s30, 0x60", ::: "s20","s21","s22","s23","s24","s25","s26","s27","s28","s29","s30")
  // 25: v_cmp -> s_and exec -> s_cbranch taken to the next line
  T("v_cmp_le_i32_e32 vcc, 0, v41\n s_and_b64 s[20:21], vcc, exec\n s_cbranch_scc1 6f\n s_nop 0\n6:", ::: "s20","s21","vcc")
  // 26: DPP min step pair (s_nop 1 + v_min_u32_dpp), the scheduler's wave reduction
  T("s_nop 1\n v_min_u32_dpp v40, v40, v40 row_shr:1 row_mask:0xf bank_mask:0xf", ::: "v40")
}

int main() {
  uint32_t *buf; uint64_t *out;
  hipMalloc(&buf, 4096); hipMemset(buf, 0, 4096);
  hipMalloc(&out, 64 * 8); hipMemset(out, 0, 64 * 8);
  const char *names[] = {"empty", "s_load_x4+wait", "ds_read_b32+wait", "ds_read_b128 bcast+wait",
    "s_load+ds_read+wait", "s_add dep", "2x s_add indep", "v_add dep", "s_branch taken",
    "s_cmp+cbranch not taken", "getpc+add+addc+setpc", "readfirstlane->s_add", "global_load_x4+wait",
    "2x(s_load_x2+wait)", "ds_read x2+wait+v_add+ds_write", "v_add addr + ds_read + wait",
    "s_and+s_lshr", "2x s_mov_b64", "s_cmp+cbranch taken", "ds_write_b32", "s_load_x8+wait",
    "4x readfirstlane + s_and", "v_cmp+s_and+cbranch nt", "rfl+nop+v_cmp_ne+s_and+cbr",
    "12 SALU (transfer checks)", "v_cmp+s_and+cbranch taken", "s_nop1 + v_min_dpp"};
  for (int it = 0; it < 3; it++) {
    hipLaunchKernelGGL(kbench, dim3(1), dim3(64), 0, 0, buf, out);
    hipDeviceSynchronize();
  }
  uint64_t h[64];
  hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
  for (int i = 0; i < 27; i++)
    printf("%2d %-34s %8.1f cyc/rep (memtime ticks)\n", i, names[i], (double)(h[i] - h[0]) / 64.0);
  // the memtime clock rate
  int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeClockRate, 0);
  printf("device clock attr %d kHz\n", rate);
  return 0;
}
