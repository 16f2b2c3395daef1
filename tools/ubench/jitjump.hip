// jitjump.hip -- feasibility probe for per-module code generation: a kernel built by
// hipcc jumps (s_setpc_b64) into a code block that hiprtc compiled at run time and
// hipModuleLoadData loaded, and the block jumps back. Prints "jit ok" when every lane
// saw the block's effect.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/jitjump tools/ubench/jitjump.hip -lhiprtc
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdio>
#include <vector>

#define CK(x) do { auto _e = (x); if (_e != hipSuccess) { printf("%s: %d\n", #x, (int)_e); return 1; } } while (0)

// the run-time source: one block at a label, and a kernel that reports its address
static const char *kSrc = R"(
extern "C" __global__ void wbjit_addrs(unsigned long long *out) {
  unsigned lo, hi;
  asm volatile("s_getpc_b64 s[6:7]\n"
               "Lpc_%=:\n"
               "s_add_u32 s6, s6, Lblk_%= - Lpc_%=\n"
               "s_addc_u32 s7, s7, 0\n"
               "s_mov_b32 %0, s6\n"
               "s_mov_b32 %1, s7\n"
               "s_branch Lskip_%=\n"
               ".p2align 8\n"
               "Lblk_%=:\n"
               "v_add_u32_e32 v120, 41, v120\n"
               "v_mul_lo_u32 v120, v120, 3\n"
               "s_setpc_b64 s[66:67]\n"
               "Lskip_%=:\n" : "=s"(lo), "=s"(hi) : : "s6", "s7", "scc");
  if (threadIdx.x == 0) out[0] = ((unsigned long long)hi << 32) | lo;
}
)";

__global__ void caller(unsigned *data, unsigned long long target) {
  const unsigned lo = (unsigned)target, hi = (unsigned)(target >> 32);
  unsigned v = data[threadIdx.x];
  asm volatile("v_mov_b32 v120, %[v]\n\t"
               "s_mov_b32 s68, %[lo]\n\t"
               "s_mov_b32 s69, %[hi]\n\t"
               "s_getpc_b64 s[66:67]\n"
               "Lret_%=:\n\t"
               "s_add_u32 s66, s66, Lback_%= - Lret_%=\n\t"
               "s_addc_u32 s67, s67, 0\n\t"
               "s_setpc_b64 s[68:69]\n"
               "Lback_%=:\n\t"
               "v_mov_b32 %[v], v120"
               : [v] "+v"(v)
               : [lo] "s"(lo), [hi] "s"(hi)
               : "v120", "s66", "s67", "s68", "s69", "scc");
  data[threadIdx.x] = v;
}

int main() {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, kSrc, "wbjit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) return 1;
  const char *opts[] = {"--offload-arch=gfx950", "-O2"};
  if (hiprtcCompileProgram(prog, 2, opts) != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::vector<char> log(n + 1);
    hiprtcGetProgramLog(prog, log.data());
    printf("compile failed:\n%s\n", log.data());
    return 1;
  }
  size_t sz = 0;
  hiprtcGetCodeSize(prog, &sz);
  std::vector<char> code(sz);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  hipModule_t mod;
  CK(hipModuleLoadData(&mod, code.data()));
  hipFunction_t fn;
  CK(hipModuleGetFunction(&fn, mod, "wbjit_addrs"));
  unsigned long long *daddr;
  CK(hipMalloc(&daddr, 8));
  void *args[] = {&daddr};
  CK(hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, nullptr, args, nullptr));
  unsigned long long addr = 0;
  CK(hipMemcpy(&addr, daddr, 8, hipMemcpyDeviceToHost));
  printf("block at 0x%llx (code object %zu bytes)\n", addr, sz);
  unsigned *d;
  std::vector<unsigned> h(64);
  for (int i = 0; i < 64; i++) h[i] = i;
  CK(hipMalloc(&d, 256));
  CK(hipMemcpy(d, h.data(), 256, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(caller, dim3(1), dim3(64), 0, 0, d, addr);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h.data(), d, 256, hipMemcpyDeviceToHost));
  bool ok = true;
  for (int i = 0; i < 64; i++) ok &= h[i] == (unsigned)(i + 41) * 3u;
  printf(ok ? "jit ok\n" : "jit MISMATCH\n");
  return ok ? 0 : 2;
}
