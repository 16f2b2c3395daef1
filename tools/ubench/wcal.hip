// Write-back calibration for the counters behind C3's HBM figure (tuning aid only): how
// many bytes WRITE_SIZE / FETCH_SIZE report for known access patterns in the interpreter's
// linear-memory layout -- 64 lanes of a wave interleaved in 128-byte granules, a lane's
// consecutive granules 8 KiB apart. 1024 waves x 64 lanes (C3's 64K instances), 16 KiB per
// lane (1 GiB). Run each kernel under rocprofv3 --pmc WRITE_SIZE (and FETCH_SIZE) and
// divide by the bytes each writes (printed).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

constexpr uint32_t kWaves = 1024, kRows = 128;             // 128 granules of 128 B per lane
constexpr size_t kWaveWords = size_t(kRows) * 64 * 32;     // words per wave region
constexpr size_t kWords = kWaves * kWaveWords;             // 1 GiB

__device__ __forceinline__ uint32_t *gran(uint32_t *m, uint32_t wave, uint32_t lane, uint32_t row) {
  return m + wave * kWaveWords + (size_t(row) * 64 + lane) * 32;
}

// 16 B per lane, coalesced, every word once (the guide's calibration access)
__global__ void k_stream_read(const uint4 *m, uint32_t *out) {
  uint32_t x = 0;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < kWords / 4; i += gridDim.x * blockDim.x) {
    const uint4 v = m[i];
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) out[0] = x;
}
__global__ void k_stream_write(uint4 *m) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < kWords / 4; i += gridDim.x * blockDim.x)
    m[i] = make_uint4(i, i, i, i);
}
// one dword per granule (an isolated 4-byte store per 128-byte line)
__global__ void k_one_per_line(uint32_t *m) {
  const uint32_t wave = blockIdx.x, lane = threadIdx.x;
  for (uint32_t r = 0; r < kRows; r++) gran(m, wave, lane, r)[(r * 7) & 31] = r;
}
// every dword of each granule, one store instruction per dword, granule by granule
__global__ void k_dense_seq(uint32_t *m) {
  const uint32_t wave = blockIdx.x, lane = threadIdx.x;
  for (uint32_t r = 0; r < kRows; r++)
    for (uint32_t w = 0; w < 32; w++) gran(m, wave, lane, r)[w] = r + w;
}
// every other dword of each granule (a Hoare scan's swap stores at density 1/2)
__global__ void k_half_seq(uint32_t *m) {
  const uint32_t wave = blockIdx.x, lane = threadIdx.x;
  for (uint32_t r = 0; r < kRows; r++)
    for (uint32_t w = 0; w < 32; w += 2) gran(m, wave, lane, r)[w] = r + w;
}
// every dword of each granule, but a granule's stores spread over the whole kernel (word
// w of every granule, then word w + 1 ...): a line is revisited after 1 GiB / 32 of stores
__global__ void k_dense_spread(uint32_t *m) {
  const uint32_t wave = blockIdx.x, lane = threadIdx.x;
  for (uint32_t w = 0; w < 32; w++)
    for (uint32_t r = 0; r < kRows; r++) gran(m, wave, lane, r)[w] = r + w;
}
// a read-modify-write walk like a Hoare scan: read every dword of a granule in order,
// store to every other one just after reading it
__global__ void k_scan_swap(uint32_t *m) {
  const uint32_t wave = blockIdx.x, lane = threadIdx.x;
  for (uint32_t r = 0; r < kRows; r++) {
    uint32_t *g = gran(m, wave, lane, r);
    for (uint32_t w = 0; w < 32; w++) {
      const uint32_t v = __builtin_nontemporal_load(&g[w]) * 3u + 1u;
      if (w & 1) g[w - 1] = v;
    }
  }
}

// read every dword of granule r, store to every other dword of granule r - gap (read gap
// granules earlier): how long a line read into L2 keeps taking stores without a write miss
template <uint32_t kGap>
__global__ void k_scan_swap_gap(uint32_t *m) {
  const uint32_t wave = blockIdx.x, lane = threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t r = 0; r < kRows + kGap; r++) {
    if (r < kRows) {
      const uint32_t *g = gran(m, wave, lane, r);
      for (uint32_t w = 0; w < 32; w++) acc += g[w];   // (plain loads, as the compiled runs issue)
    }
    if (r >= kGap) {
      uint32_t *s = gran(m, wave, lane, r - kGap);
      for (uint32_t w = 0; w < 32; w += 2) s[w] = acc + w;
    }
  }
}
// stores only, but to granules the previous kernel just read (is the L2 still holding them?)
__global__ void k_read_all(const uint32_t *m, uint32_t *out) {
  const uint32_t wave = blockIdx.x, lane = threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t r = 0; r < kRows; r++)
    for (uint32_t w = 0; w < 32; w += 8) acc += gran(const_cast<uint32_t *>(m), wave, lane, r)[w];
  if (acc == 0x1234567u) out[0] = acc;
}

int main(int argc, char **argv) {
  uint32_t *m = nullptr, *out = nullptr;
  if (hipMalloc(&m, kWords * 4) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(m, 0, kWords * 4);
  (void)hipDeviceSynchronize();
  const char *only = argc > 1 ? argv[1] : nullptr;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](const char *name, double bytes, auto launch) {
    if (only && strcmp(only, name)) return;
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-16s bytes %.6g  %.3f ms  %.1f GB/s\n", name, bytes, ms, bytes / ms / 1e6);
  };
  const dim3 g(kWaves), b(64);
  run("stream_read", double(kWords) * 4, [&] { k_stream_read<<<8192, 256>>>((const uint4 *)m, out); });
  run("stream_write", double(kWords) * 4, [&] { k_stream_write<<<8192, 256>>>((uint4 *)m); });
  run("one_per_line", double(kWaves) * 64 * kRows * 4, [&] { k_one_per_line<<<g, b>>>(m); });
  run("dense_seq", double(kWords) * 4, [&] { k_dense_seq<<<g, b>>>(m); });
  run("half_seq", double(kWords) * 2, [&] { k_half_seq<<<g, b>>>(m); });
  run("dense_spread", double(kWords) * 4, [&] { k_dense_spread<<<g, b>>>(m); });
  run("scan_swap", double(kWords) * 2, [&] { k_scan_swap<<<g, b>>>(m); });
  run("gap1", double(kWords) * 2, [&] { k_scan_swap_gap<1><<<g, b>>>(m); });
  run("gap4", double(kWords) * 2, [&] { k_scan_swap_gap<4><<<g, b>>>(m); });
  run("gap16", double(kWords) * 2, [&] { k_scan_swap_gap<16><<<g, b>>>(m); });
  run("gap64", double(kWords) * 2, [&] { k_scan_swap_gap<64><<<g, b>>>(m); });
  run("read_all", 0, [&] { k_read_all<<<g, b>>>(m, out); });
  return 0;
}
