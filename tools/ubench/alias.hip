// L2 set aliasing between waves (tuning aid only): C3's Hoare partitions in miniature.
// 1024 waves x 64 lanes; every lane sweeps two pointers through its own words (i up, j
// down, 1-2 words a step, a load and a store at each, the next step depending on the
// loaded words), in the interpreter's layout: 128-byte granules interleaved over a wave's
// 64 lanes, waves `stride` bytes apart. The reserved layout puts waves rpages x 4 MiB
// apart (68 MiB for C3's 17 pages): every wave's lines at the same offset then share the
// low 22 address bits. Run under rocprofv3 --pmc WRITE_SIZE (and --kernel-trace): one
// dispatch per stride, in the order printed.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr uint32_t kWaves = 1024;

__global__ void __launch_bounds__(64) k_sweep(uint32_t *m, size_t stride_words, uint32_t n_words,
                                               uint32_t rounds, uint32_t *out, uint32_t desync) {
  const uint32_t wave = blockIdx.x, lane = threadIdx.x;
  uint32_t *base = m + wave * stride_words + lane * 32;
  auto at = [&](uint32_t w) { return base + size_t(w >> 5) * 2048 + (w & 31); };
  uint32_t x = lane * 2654435761u + wave + 1;
  // desync: every lane starts at its own point of the sweep (lanes apart, as C3's are)
  uint32_t i = desync ? (x >> 8) % (n_words / 2) : 0, j = desync ? i + n_words / 2 : n_words - 1;
  for (uint32_t r = 0; r < rounds; r++) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    i += 1 + (x & 1);
    j -= 1 + ((x >> 1) & 1);
    if (i >= j) { i = 0; j = n_words - 1; }
    const uint32_t a = *at(i), b = *at(j);
    *at(i) = b ^ x;
    *at(j) = a + x;
    x ^= a ^ b;
  }
  if (x == 0x12345u) out[0] = x;
}

int main(int argc, char **argv) {
  const uint32_t n_words = argc > 1 ? atoi(argv[1]) : 4096;      // words swept per lane
  const uint32_t rounds = argc > 2 ? atoi(argv[2]) : 4000;
  const uint32_t waves = argc > 3 ? atoi(argv[3]) : kWaves;       // (fewer: a smaller L2 footprint)
  const size_t s0 = size_t(17) << 22;                             // 68 MiB (17 pages x 4 MiB)
  const size_t strides[] = {s0, size_t(n_words) * 256};
  uint32_t *m, *out;
  size_t most = 0;
  for (size_t s : strides) most = s > most ? s : most;
  if (hipMalloc(&m, most * kWaves + (1 << 20)) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(m, 0, most * kWaves);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (uint32_t desync = 0; desync < 2; desync++)
  for (size_t s : strides) {
    k_sweep<<<waves, 64>>>(m, s / 4, n_words, rounds / 8, out, desync);   // (warm the pages)
    hipEventRecord(e0);
    k_sweep<<<waves, 64>>>(m, s / 4, n_words, rounds, out, desync);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("desync %u waves %u stride %zu B (%+lld from 68 MiB): %.3f ms, %.1f ns per step; stores %.4g B\n",
           desync, waves, s, (long long)s - (long long)s0, ms, ms * 1e6 / rounds, 8.0 * rounds * 64 * waves);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
