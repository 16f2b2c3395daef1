// multi.cpp -- one batch over several devices from one process (SURVEY.md §8(b) NumDevices,
// §8(e)): WasmEdge_BatchConfigure::Devices / DeviceCount / Partition.
//
// The reference runs concurrent executes inside one process: VM::execute takes a shared lock
// (include/vm/vm.h:137-141) and async executes run on their own threads (include/vm/async.h:
// 25-40). Here the instances themselves are split: the parent context holds one shard per
// entry of Devices -- a whole single-device context over its part of the instance ids --
// and routes every call. Batch-wide calls (SetArgs, Reset, Run, Results, hashes, costs) go
// to every shard, Reset and Run on one host thread per shard (each shard has its own stream,
// so shards on one device overlap too); per-instance calls go to the instance's shard.
// Instances share nothing, so there is no collective: the gather of per-instance outputs is
// a host-side scatter into the caller's [NumInstances] arrays.
#include <algorithm>
#include <thread>
#include <vector>

#include "batch_ctx.h"
#include "multi.h"

namespace wbh {

// Blocks: whole waves, ceil(waves / G) per shard in id order; interleave: id mod G.
static uint32_t block_span(uint32_t n, uint32_t g_count) {
  const uint32_t waves = (n + 63) / 64, q = (waves + g_count - 1) / g_count;
  return q * 64;
}

bool placement(uint32_t n, uint32_t g_count, uint32_t part, uint32_t inst, uint32_t *g,
               uint32_t *local) {
  if (g_count == 0 || inst >= n || part > WASMEDGE_BATCH_PARTITION_INTERLEAVE) return false;
  if (part == WASMEDGE_BATCH_PARTITION_INTERLEAVE) {
    *g = inst % g_count;
    *local = inst / g_count;
  } else {
    const uint32_t span = block_span(n, g_count);
    *g = inst / span;
    *local = inst % span;
  }
  return true;
}

uint32_t shard_size(uint32_t n, uint32_t g_count, uint32_t part, uint32_t g) {
  if (part == WASMEDGE_BATCH_PARTITION_INTERLEAVE) return g < n ? (n - g + g_count - 1) / g_count : 0;
  const uint64_t span = block_span(n, g_count), lo = std::min<uint64_t>(n, g * span),
                 hi = std::min<uint64_t>(n, (g + 1) * span);
  return uint32_t(hi - lo);
}

}  // namespace wbh

uint32_t WasmEdge_BatchContext::gid(uint32_t local) const {
  if (!parent) return local;
  const uint32_t G = uint32_t(parent->shards.size());
  if (parent->part == WASMEDGE_BATCH_PARTITION_INTERLEAVE) return local * G + shard_g;
  return shard_g * wbh::block_span(parent->n, G) + local;
}

namespace wbm {

using wbh::R;
using Ctx = WasmEdge_BatchContext;

namespace {

// every shard in turn, stopping at the first failure (its code; its message becomes the
// parent's last error)
template <class F>
WasmEdge_Result each(Ctx *C, F f) {
  for (Ctx *s : C->shards) {
    if (!s) continue;
    const WasmEdge_Result r = f(s);
    if (r.Code) {
      C->last_error = s->last_error;
      return r;
    }
  }
  return R(0);
}

// every shard on a thread of its own; the first failure in shard order
template <class F>
WasmEdge_Result each_parallel(Ctx *C, F f) {
  std::vector<WasmEdge_Result> rs(C->shards.size(), R(0));
  std::vector<std::thread> th;
  for (size_t g = 0; g < C->shards.size(); g++)
    if (C->shards[g]) th.emplace_back([&, g]() { rs[g] = f(C->shards[g]); });
  for (auto &t : th) t.join();
  for (size_t g = 0; g < C->shards.size(); g++)
    if (rs[g].Code) {
      C->last_error = C->shards[g]->last_error;
      return rs[g];
    }
  return R(0);
}

// a shard's [n_g] array scattered into the batch's [n] array (element size `sz`, `per`
// elements per instance)
void scatter(const Ctx *s, const uint8_t *src, uint8_t *dst, size_t sz, size_t per) {
  for (uint32_t i = 0; i < s->n; i++)
    memcpy(dst + size_t(s->gid(i)) * per * sz, src + size_t(i) * per * sz, per * sz);
}

}  // namespace

bool route(const Ctx *C, uint32_t inst, Ctx **s, uint32_t *local) {
  uint32_t g = 0;
  if (!wbh::placement(C->n, uint32_t(C->shards.size()), C->part, inst, &g, local)) return false;
  *s = C->shards[g];
  return *s != nullptr;
}

Ctx *create(const WasmEdge_BatchConfigure &conf, const uint8_t *wasm, uint32_t len, uint32_t n,
            const WasmEdge_BatchImport *imports, uint32_t nimports, WasmEdge_Result *res) {
  const uint32_t G = conf.DeviceCount;
  if (!conf.Devices || conf.Partition > WASMEDGE_BATCH_PARTITION_INTERLEAVE) {
    wbh::g_last_create_error = "Devices must list DeviceCount ordinals; Partition 0 or 1";
    if (res) *res = R(wbh::kWrongVMWorkflow);
    return nullptr;
  }
  int caller_dev = -1;
  (void)hipGetDevice(&caller_dev);
  Ctx *P = new Ctx();
  P->conf = conf;
  P->conf.CostTable = nullptr;
  P->n = n;
  P->part = conf.Partition;
  P->shards.assign(G, nullptr);
  WasmEdge_Result r = R(0);
  for (uint32_t g = 0; g < G && !r.Code; g++) {
    const uint32_t ng = wbh::shard_size(n, G, conf.Partition, g);
    if (ng == 0) continue;
    WasmEdge_BatchConfigure cg = conf;
    cg.Devices = nullptr;
    cg.DeviceCount = 0;
    cg.DeviceOrdinal = conf.Devices[g];
    Ctx *s = WasmEdge_BatchCreateWithImports(&cg, wasm, len, ng, imports, nimports, &r);
    if (!s) break;
    s->parent = P;
    s->shard_g = g;
    if (conf.HostThreads <= 1) s->host_mu = &P->own_host_mu;
    P->shards[g] = s;
  }
  if (caller_dev >= 0) (void)hipSetDevice(caller_dev);   // (shard creation set its own)
  if (r.Code) {
    destroy(P);
    if (res) *res = r;
    return nullptr;
  }
  P->nwaves = (n + 63) / 64;
  if (res) *res = R(0);
  return P;
}

void destroy(Ctx *C) {
  for (Ctx *s : C->shards)
    if (s) WasmEdge_BatchDelete(s);
  delete C;
}

WasmEdge_Result set_args(Ctx *C, const WasmEdge_String name, const WasmEdge_Value *params,
                         uint32_t plen) {
  std::vector<WasmEdge_Value> rows;
  return each(C, [&](Ctx *s) {
    rows.assign(size_t(s->n) * plen, WasmEdge_Value{});
    for (uint32_t i = 0; i < s->n && params; i++)
      std::copy(params + size_t(s->gid(i)) * plen, params + size_t(s->gid(i) + 1) * plen,
                rows.begin() + ptrdiff_t(size_t(i) * plen));
    return WasmEdge_BatchSetArgs(s, name, plen ? rows.data() : nullptr, plen);
  });
}

// Reset / Run: every shard on its own thread; the time is the slowest shard's
WasmEdge_Result reset(Ctx *C, double *secs) {
  std::vector<double> t(C->shards.size(), 0.0);
  const WasmEdge_Result r = each_parallel(C, [&](Ctx *s) {
    return WasmEdge_BatchReset(s, secs ? &t[s->shard_g] : nullptr);
  });
  if (secs) *secs = *std::max_element(t.begin(), t.end());
  return r;
}

WasmEdge_Result run(Ctx *C, double *secs) {
  std::vector<double> t(C->shards.size(), 0.0);
  const WasmEdge_Result r = each_parallel(C, [&](Ctx *s) {
    return WasmEdge_BatchRun(s, secs ? &t[s->shard_g] : nullptr);
  });
  if (secs) *secs = *std::max_element(t.begin(), t.end());
  // one memory layout for the whole batch (batch_api.cpp layout_trial): the shards run the
  // same module through the same calls, so their trials step together and only a verdict
  // can differ; the first shard's stands for all of them
  if (!r.Code)
    if (Ctx *f = first(C))
      for (Ctx *s : C->shards)
        if (s && s != f) s->trial = f->trial;
  return r;
}

WasmEdge_Result results(Ctx *C, WasmEdge_Value *rets, uint32_t rlen, uint8_t *st, uint64_t *cnt) {
  std::vector<WasmEdge_Value> rv;
  std::vector<uint8_t> sv;
  std::vector<uint64_t> cv;
  return each(C, [&](Ctx *s) {
    rv.assign(size_t(s->n) * std::max<uint32_t>(rlen, 1), WasmEdge_Value{});
    sv.assign(s->n, 0);
    cv.assign(s->n, 0);
    const WasmEdge_Result r = WasmEdge_BatchResults(s, rets ? rv.data() : nullptr, rlen, sv.data(), cv.data());
    if (r.Code) return r;
    if (rets && rlen)
      scatter(s, reinterpret_cast<const uint8_t *>(rv.data()), reinterpret_cast<uint8_t *>(rets),
              sizeof(WasmEdge_Value), rlen);
    if (st) scatter(s, sv.data(), st, 1, 1);
    if (cnt) scatter(s, reinterpret_cast<const uint8_t *>(cv.data()), reinterpret_cast<uint8_t *>(cnt), 8, 1);
    return R(0);
  });
}

// [n] u64 outputs (hashes, costs)
WasmEdge_Result gather_u64(Ctx *C, uint64_t *out, WasmEdge_Result (*f)(Ctx *, uint64_t *)) {
  std::vector<uint64_t> v;
  return each(C, [&](Ctx *s) {
    v.assign(s->n, 0);
    const WasmEdge_Result r = f(s, v.data());
    if (!r.Code) scatter(s, reinterpret_cast<const uint8_t *>(v.data()), reinterpret_cast<uint8_t *>(out), 8, 1);
    return r;
  });
}

}  // namespace wbm

extern "C" {

WasmEdge_Result WasmEdge_BatchPlacement(uint32_t NumInstances, uint32_t DeviceCount, uint32_t Partition,
                                        uint32_t Inst, uint32_t *Shard, uint32_t *Local) {
  uint32_t g = 0, l = 0;
  if (!wbh::placement(NumInstances, DeviceCount, Partition, Inst, &g, &l)) return wbh::R(wbh::kWrongVMWorkflow);
  if (Shard) *Shard = g;
  if (Local) *Local = l;
  return wbh::R(0);
}

}  // extern "C"
