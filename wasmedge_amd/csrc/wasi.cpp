// wasi.cpp -- the built-in WASI subset on the host-import yield path (wasi_impl.h holds
// the functions). WasmEdge_BatchInitWASI binds every import of wasi_snapshot_preview1
// that the subset has, with the right signature, as if the caller had registered each
// one through WasmEdge_BatchAddHostFunction -- the batched form of
// WasmEdge_ImportObjectCreateWASI / InitWASI (include/api/wasmedge/wasmedge.h:2719-2754).
#include <algorithm>

#include "batch_ctx.h"
#include "multi.h"

using namespace wbh;

namespace {

// one instance's memory through the service round's view (batch_ctx.h WaveView)
struct CtxMem final : wbw::MemIO {
  WasmEdge_BatchMemoryContext *mc;
  explicit CtxMem(WasmEdge_BatchMemoryContext *m) : mc(m) {}
  bool present() override { return mc->ctx->prog.has_mem; }
  uint64_t size() override { return mem_size(mc); }
  bool read(uint32_t off, uint32_t len, uint8_t *dst) override {
    return WasmEdge_BatchMemoryGetData(mc, dst, off, len).Code == 0;
  }
  bool write(uint32_t off, uint32_t len, const uint8_t *src) override {
    return WasmEdge_BatchMemorySetData(mc, src, off, len).Code == 0;
  }
};

WasmEdge_Result wasi_trampoline(void *Data, WasmEdge_BatchMemoryContext *M,
                                const WasmEdge_Value *Params, WasmEdge_Value *Returns) {
  const auto *slot = static_cast<const WasmEdge_BatchContext::WasiSlot *>(Data);
  WasmEdge_BatchContext *C = slot->ctx;
  const uint32_t inst = M->inst;   // (this context's own lane index: its WASI state)
  uint64_t a[wbw::kMaxArgs] = {0};
  uint32_t ret = 0;
  const size_t f = size_t(slot - C->wasi_slots.data());   // the import's function index
  const wb::FuncType &t = C->prog.types[C->prog.funcs[f].type];
  for (size_t k = 0; k < t.params.size() && k < wbw::kMaxArgs; k++)
    a[k] = t.params[k] == 0x7E ? uint64_t(Params[k].Value) : uint64_t(uint32_t(Params[k].Value));
  CtxMem mem(M);
  const uint8_t e = wbw::call(slot->fn, C->wasi_env, C->wasi_lanes[inst], mem, a, &ret);
  if (e) return R(e);
  if (!t.results.empty()) Returns[0].Value = ret;
  return R(0);
}

}  // namespace

extern "C" {

WasmEdge_Result WasmEdge_BatchInitWASI(WasmEdge_BatchContext *C, const char *const *Args,
                                       const uint32_t ArgLen, const char *const *Envs,
                                       const uint32_t EnvLen) {
  return WasmEdge_BatchInitWASIWithPreopens(C, Args, ArgLen, Envs, EnvLen, nullptr, 0);
}

WasmEdge_Result WasmEdge_BatchInitWASIWithPreopens(WasmEdge_BatchContext *C, const char *const *Args,
                                                   const uint32_t ArgLen, const char *const *Envs,
                                                   const uint32_t EnvLen,
                                                   const char *const *Preopens,
                                                   const uint32_t PreopenLen) {
  if (!C) return R(kWrongVMWorkflow);
  if (!C->shards.empty()) {
    const uint64_t seed = wbw::host_seed();
    const WasmEdge_Result r = wbm::all(C, [&](WasmEdge_BatchContext *s) {
      return WasmEdge_BatchInitWASIWithPreopens(s, Args, ArgLen, Envs, EnvLen, Preopens, PreopenLen);
    });
    if (r.Code) return r;
    // (one seed, and every lane's generator keyed on its id in the whole batch)
    for (uint32_t i = 0; i < C->n; i++) {
      WasmEdge_BatchContext *s;
      uint32_t l;
      if (!wbm::route(C, i, &s, &l)) continue;
      s->wasi_env.seed = seed;
      s->wasi_lanes[l].index = i;
    }
    return r;
  }
  C->wasi_env.args.clear();
  C->wasi_env.envs.clear();
  C->wasi_env.preopens.clear();
  C->wasi_env.host.clear();
  C->wasi_env.fixed_clock = false;
  C->wasi_env.seed = wbw::host_seed();
  for (uint32_t k = 0; k < ArgLen; k++) C->wasi_env.args.emplace_back(Args && Args[k] ? Args[k] : "");
  for (uint32_t k = 0; k < EnvLen; k++) C->wasi_env.envs.emplace_back(Envs && Envs[k] ? Envs[k] : "");
  // "guest:host" or one path for both (environ.cpp:57-66); the fds follow the list's order
  for (uint32_t k = 0; k < PreopenLen; k++) wbw::add_preopen(C->wasi_env, Preopens && Preopens[k] ? Preopens[k] : "");
  C->wasi_lanes.assign(C->n, wbw::Lane{});
  for (uint32_t i = 0; i < C->n; i++) C->wasi_lanes[i].index = i;
  const wb::Program &P = C->prog;
  C->wasi_slots.assign(P.funcs.size(), WasmEdge_BatchContext::WasiSlot{C, -1});
  for (uint32_t f = 0; f < P.n_imported; f++) {
    if (P.funcs[f].import_module != "wasi_snapshot_preview1") continue;
    const wb::FuncType &t = P.types[P.funcs[f].type];
    const int fn = wbw::lookup(P.funcs[f].import_name, t.params, t.results);
    if (fn < 0) continue;
    C->wasi_slots[f].fn = fn;
    C->hosts[f] = WasmEdge_BatchContext::HostFn{wasi_trampoline, &C->wasi_slots[f]};
  }
  return R(0);
}

WasmEdge_Result WasmEdge_BatchWASISetDeterministic(WasmEdge_BatchContext *C, uint64_t Seed,
                                                   uint64_t ClockNs) {
  if (!C) return R(kWrongVMWorkflow);
  if (!C->shards.empty())
    return wbm::all(C, [&](WasmEdge_BatchContext *s) { return WasmEdge_BatchWASISetDeterministic(s, Seed, ClockNs); });
  C->wasi_env.seed = Seed;
  C->wasi_env.fixed_clock = true;
  C->wasi_env.clock_ns = ClockNs;
  for (auto &L : C->wasi_lanes) {   // (the lanes' tables and generators start over)
    L.fs_ready = false;
    L.fds.clear();
    L.clock_calls = 0;
  }
  return R(0);
}

WasmEdge_Result WasmEdge_BatchWASISetInstanceArgs(WasmEdge_BatchContext *C, uint32_t Inst,
                                                  const char *const *Args, const uint32_t ArgLen) {
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (C && !C->shards.empty())
    return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchWASISetInstanceArgs(s, l, Args, ArgLen)
                                       : R(kWrongVMWorkflow);
  if (!C || Inst >= C->wasi_lanes.size()) return R(kWrongVMWorkflow);
  wbw::Lane &L = C->wasi_lanes[Inst];
  L.own_args = true;
  L.args.clear();
  for (uint32_t k = 0; k < ArgLen; k++) L.args.emplace_back(Args && Args[k] ? Args[k] : "");
  return R(0);
}

uint32_t WasmEdge_BatchWASIGetExitCode(const WasmEdge_BatchContext *C, uint32_t Inst) {
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (C && !C->shards.empty()) return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchWASIGetExitCode(s, l) : 0;
  if (!C || Inst >= C->wasi_lanes.size()) return 0;
  return C->wasi_lanes[Inst].exit_code;
}

uint32_t WasmEdge_BatchWASIGetOutput(const WasmEdge_BatchContext *C, uint32_t Inst, uint32_t Fd,
                                     uint8_t *Buf, uint32_t Len) {
  WasmEdge_BatchContext *sh;
  uint32_t l;
  if (C && !C->shards.empty()) return wbm::route(C, Inst, &sh, &l) ? WasmEdge_BatchWASIGetOutput(sh, l, Fd, Buf, Len) : 0;
  if (!C || Inst >= C->wasi_lanes.size() || (Fd != 1 && Fd != 2)) return 0;
  const std::string &s = C->wasi_lanes[Inst].out[Fd - 1];
  if (Buf) memcpy(Buf, s.data(), std::min<size_t>(Len, s.size()));
  return uint32_t(s.size());
}

}  // extern "C"
