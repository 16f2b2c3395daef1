// Probe of the HIP virtual-memory API on the box (tuning / design aid only): can linear
// memory be a large VA reservation whose 4 MiB wave rows are committed on demand, as the
// reference's mmap'd reservation is (lib/system/allocator.cpp:60-142)? Reserves a VA range,
// maps physical rows at scattered offsets, writes and reads them from a kernel, measures
// the host cost of one map + access call, then unmaps and frees.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <chrono>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("FAIL %s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_fill(uint32_t *p, size_t words, uint32_t tag) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < words; i += gridDim.x * blockDim.x) p[i] = uint32_t(i) ^ tag;
}
__global__ void k_check(const uint32_t *p, size_t words, uint32_t tag, uint32_t *bad) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < words; i += gridDim.x * blockDim.x)
    if (p[i] != (uint32_t(i) ^ tag)) atomicAdd(bad, 1u);
}

int main() {
  int dev = 0;
  CK(hipGetDevice(&dev));
  int vmm = 0;
  (void)hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, dev);
  printf("VirtualMemoryManagementSupported = %d\n", vmm);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  size_t rec = 0;
  CK(hipMemGetAllocationGranularity(&rec, &prop, hipMemAllocationGranularityRecommended));
  printf("granularity min %zu recommended %zu\n", gran, rec);
  const size_t row = size_t(4) << 20;   // one wave's page: 64 lanes x 64 KiB
  for (size_t tib : {1, 16, 64}) {
    void *va = nullptr;
    const size_t span = tib << 40;
    hipError_t e = hipMemAddressReserve(&va, span, 0, nullptr, 0);
    printf("reserve %zu TiB: %s %p\n", tib, hipGetErrorString(e), va);
    if (e == hipSuccess) (void)hipMemAddressFree(va, span);
  }
  const size_t span = size_t(16) << 40;
  void *va = nullptr;
  CK(hipMemAddressReserve(&va, span, 0, nullptr, 0));
  std::vector<hipMemGenericAllocationHandle_t> hs;
  std::vector<size_t> offs = {0, row * 17, (size_t(1) << 36) + row * 3, span - row};
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  double map_us = 0;
  for (size_t off : offs) {
    hipMemGenericAllocationHandle_t h;
    const auto t0 = std::chrono::steady_clock::now();
    CK(hipMemCreate(&h, row, &prop, 0));
    CK(hipMemMap((char *)va + off, row, 0, h, 0));
    CK(hipMemSetAccess((char *)va + off, row, &acc, 1));
    map_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    hs.push_back(h);
  }
  printf("create+map+access per 4 MiB row: %.1f us\n", map_us / offs.size());
  uint32_t *bad = nullptr;
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  for (size_t k = 0; k < offs.size(); k++) {
    uint32_t *p = (uint32_t *)((char *)va + offs[k]);
    k_fill<<<256, 256>>>(p, row / 4, uint32_t(k * 0x9E3779B9u));
    k_check<<<256, 256>>>(p, row / 4, uint32_t(k * 0x9E3779B9u), bad);
  }
  CK(hipDeviceSynchronize());
  uint32_t nbad = 0;
  CK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
  // host copies through the mapping (the service rounds' views use hipMemcpy2D)
  std::vector<uint32_t> h(1024);
  CK(hipMemcpy(h.data(), (char *)va + offs[2], 4096, hipMemcpyDeviceToHost));
  printf("kernel check: %u bad words; host read word 5 = %08x (expect %08x)\n", nbad, h[5],
         5u ^ uint32_t(2 * 0x9E3779B9u));
  // memset of a mapped row (Reset zeroes handed-out rows)
  CK(hipMemset((char *)va + offs[1], 0, row));
  CK(hipDeviceSynchronize());
  for (size_t k = 0; k < offs.size(); k++) {
    CK(hipMemUnmap((char *)va + offs[k], row));
    CK(hipMemRelease(hs[k]));
  }
  // steady-state costs per phase: 64 rows one by one, then one 1 GiB chunk
  {
    using clk = std::chrono::steady_clock;
    double tc = 0, tm = 0, ta = 0, tu = 0;
    std::vector<hipMemGenericAllocationHandle_t> h64(64);
    for (int k = 0; k < 64; k++) {
      char *p = (char *)va + (size_t(k) << 30);
      auto t0 = clk::now();
      CK(hipMemCreate(&h64[k], row, &prop, 0));
      auto t1 = clk::now();
      CK(hipMemMap(p, row, 0, h64[k], 0));
      auto t2 = clk::now();
      CK(hipMemSetAccess(p, row, &acc, 1));
      auto t3 = clk::now();
      tc += std::chrono::duration<double, std::micro>(t1 - t0).count();
      tm += std::chrono::duration<double, std::micro>(t2 - t1).count();
      ta += std::chrono::duration<double, std::micro>(t3 - t2).count();
    }
    for (int k = 0; k < 64; k++) {
      auto t0 = clk::now();
      CK(hipMemUnmap((char *)va + (size_t(k) << 30), row));
      CK(hipMemRelease(h64[k]));
      tu += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    }
    printf("per 4 MiB row (64 rows): create %.1f us, map %.1f us, access %.1f us, unmap+release %.1f us\n",
           tc / 64, tm / 64, ta / 64, tu / 64);
    const size_t big = size_t(1) << 30;
    hipMemGenericAllocationHandle_t hb;
    auto t0 = clk::now();
    CK(hipMemCreate(&hb, big, &prop, 0));
    CK(hipMemMap(va, big, 0, hb, 0));
    CK(hipMemSetAccess(va, big, &acc, 1));
    const double tb = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
    CK(hipMemset(va, 0, big));
    CK(hipDeviceSynchronize());
    CK(hipMemUnmap(va, big));
    CK(hipMemRelease(hb));
    printf("one 1 GiB chunk: create+map+access %.1f us\n", tb);
  }
  // 2D copies over mapped rows a large pitch apart (the host service round's RoundCache:
  // one row of every wave, the waves `pitch` apart)
  {
    int maxpitch = 0;
    (void)hipDeviceGetAttribute(&maxpitch, hipDeviceAttributeMaxPitch, dev);
    printf("hipDeviceAttributeMaxPitch = %d\n", maxpitch);
    for (size_t pitch : {size_t(1) << 30, size_t(3) << 30, size_t(32) << 30}) {
      std::vector<hipMemGenericAllocationHandle_t> hh(4);
      for (int k = 0; k < 4; k++) {
        char *p = (char *)va + k * pitch;
        CK(hipMemCreate(&hh[k], row, &prop, 0));
        CK(hipMemMap(p, row, 0, hh[k], 0));
        CK(hipMemSetAccess(p, row, &acc, 1));
        k_fill<<<64, 256>>>((uint32_t *)p, 4096, uint32_t(k));
      }
      CK(hipDeviceSynchronize());
      std::vector<uint32_t> hb(4 * 4096, 0);
      hipError_t e = hipMemcpy2D(hb.data(), 4096 * 4, va, pitch, 4096 * 4, 4, hipMemcpyDeviceToHost);
      uint32_t bad = 0;
      for (int k = 0; k < 4 && e == hipSuccess; k++)
        for (uint32_t i = 0; i < 4096; i++) bad += hb[k * 4096 + i] != (i ^ uint32_t(k));
      e = e == hipSuccess ? hipMemcpy2D(va, pitch, hb.data(), 4096 * 4, 4096 * 4, 4, hipMemcpyHostToDevice) : e;
      printf("2D copy, pitch %zu GiB: %s, %u bad words\n", pitch >> 30, hipGetErrorString(e), bad);
      (void)hipGetLastError();
      CK(hipDeviceSynchronize());
      for (int k = 0; k < 4; k++) {
        CK(hipMemUnmap((char *)va + k * pitch, row));
        CK(hipMemRelease(hh[k]));
      }
    }
  }
  // adjacent commits like batch_api.cpp vm_commit: [0,2), [2,8), [8,98), [98,195) rows of
  // 4 MiB, each SetAccess'ed and zeroed with hipMemsetAsync on a non-blocking stream (or
  // hipMemset, or a kernel) -- which call refuses what
  {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const uint32_t cuts[] = {0, 2, 8, 98, 195, 196, 200};
    std::vector<std::pair<void *, size_t>> maps;
    std::vector<hipMemGenericAllocationHandle_t> hh;
    for (int mode = 0; mode < 3; mode++) {
      for (size_t k = 0; k + 1 < sizeof cuts / sizeof cuts[0]; k++) {
        const size_t bytes = size_t(cuts[k + 1] - cuts[k]) * row;
        char *at = (char *)va + (size_t(mode) << 34) + size_t(cuts[k]) * row;
        hipMemGenericAllocationHandle_t h;
        hipError_t e1 = hipMemCreate(&h, bytes, &prop, 0);
        hipError_t e2 = e1 == hipSuccess ? hipMemMap(at, bytes, 0, h, 0) : e1;
        hipError_t e3 = e2 == hipSuccess ? hipMemSetAccess(at, bytes, &acc, 1) : e2;
        hipError_t e4 = hipErrorUnknown;
        if (e3 == hipSuccess) {
          if (mode == 0) e4 = hipMemsetAsync(at, 0, bytes, st);
          else if (mode == 1) e4 = hipMemset(at, 0, bytes);
          else { k_fill<<<256, 256, 0, st>>>((uint32_t *)at, bytes / 4, 0); e4 = hipGetLastError(); }
          hipError_t e5 = hipStreamSynchronize(st);
          if (e4 == hipSuccess) e4 = e5;
        }
        printf("mode %d rows [%u,%u) at +%zu MiB: create %s map %s access %s zero %s\n", mode, cuts[k], cuts[k + 1],
               (size_t(cuts[k]) * row) >> 20, hipGetErrorString(e1), hipGetErrorString(e2), hipGetErrorString(e3),
               hipGetErrorString(e4));
        (void)hipGetLastError();
        if (e2 == hipSuccess) maps.emplace_back(at, bytes);
        if (e1 == hipSuccess) hh.push_back(h);
      }
    }
    CK(hipDeviceSynchronize());
    for (auto &m : maps) (void)hipMemUnmap(m.first, m.second);
    for (auto &h : hh) (void)hipMemRelease(h);
    (void)hipStreamDestroy(st);
  }
  // strategies for adjacent commits (which SetAccess call works), each verified by a
  // kernel fill + check of every committed row before anything else touches it:
  //  S2: SetAccess over the wave's whole committed range [0, new end) after each map
  //  S6: one mapping + SetAccess per 4 MiB row
  for (int strat : {2, 6}) {
    const uint32_t cuts[] = {0, 2, 8, 98, 195, 196, 200};
    std::vector<std::pair<void *, size_t>> maps;
    std::vector<hipMemGenericAllocationHandle_t> hh;
    char *base = (char *)va + (size_t(4 + strat) << 34);
    bool all_ok = true;
    for (size_t k = 0; k + 1 < sizeof cuts / sizeof cuts[0]; k++) {
      hipError_t e = hipSuccess;
      if (strat == 6) {
        for (uint32_t r = cuts[k]; r < cuts[k + 1] && e == hipSuccess; r++) {
          hipMemGenericAllocationHandle_t h;
          char *at = base + size_t(r) * row;
          e = hipMemCreate(&h, row, &prop, 0);
          if (e == hipSuccess) { hh.push_back(h); e = hipMemMap(at, row, 0, h, 0); }
          if (e == hipSuccess) { maps.emplace_back(at, row); e = hipMemSetAccess(at, row, &acc, 1); }
        }
      } else {
        const size_t bytes = size_t(cuts[k + 1] - cuts[k]) * row;
        char *at = base + size_t(cuts[k]) * row;
        hipMemGenericAllocationHandle_t h;
        e = hipMemCreate(&h, bytes, &prop, 0);
        if (e == hipSuccess) { hh.push_back(h); e = hipMemMap(at, bytes, 0, h, 0); }
        if (e == hipSuccess) { maps.emplace_back(at, bytes); e = hipMemSetAccess(base, size_t(cuts[k + 1]) * row, &acc, 1); }
      }
      printf("strategy S%d rows [%u,%u): %s\n", strat, cuts[k], cuts[k + 1], hipGetErrorString(e));
      (void)hipGetLastError();
      if (e != hipSuccess) { all_ok = false; break; }
    }
    if (all_ok) {
      const size_t words = size_t(200) * row / 4;
      CK(hipMemset(bad, 0, 4));
      k_fill<<<1024, 256>>>((uint32_t *)base, words, 77u);
      k_check<<<1024, 256>>>((uint32_t *)base, words, 77u, bad);
      CK(hipDeviceSynchronize());
      uint32_t nb = 0;
      CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
      printf("strategy S%d: kernel check over 200 rows: %u bad words\n", strat, nb);
    }
    CK(hipDeviceSynchronize());
    for (auto &m : maps) (void)hipMemUnmap(m.first, m.second);
    for (auto &h : hh) (void)hipMemRelease(h);
  }
  CK(hipMemAddressFree(va, span));
  printf("vmm ok\n");
  return 0;
}
