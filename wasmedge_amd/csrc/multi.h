// multi.h -- the multi-device batch (multi.cpp): a parent context routing to its shards.
#pragma once
#include "batch_ctx.h"

namespace wbm {
WasmEdge_BatchContext *create(const WasmEdge_BatchConfigure &conf, const uint8_t *wasm, uint32_t len,
                              uint32_t n, const WasmEdge_BatchImport *imports, uint32_t nimports,
                              WasmEdge_Result *res);
void destroy(WasmEdge_BatchContext *C);
// the shard and its lane for batch instance `inst` (false: out of range / no shard)
bool route(const WasmEdge_BatchContext *C, uint32_t inst, WasmEdge_BatchContext **s, uint32_t *local);
WasmEdge_Result set_args(WasmEdge_BatchContext *C, const WasmEdge_String name,
                         const WasmEdge_Value *params, uint32_t plen);
WasmEdge_Result reset(WasmEdge_BatchContext *C, double *secs);
WasmEdge_Result run(WasmEdge_BatchContext *C, double *secs);
WasmEdge_Result results(WasmEdge_BatchContext *C, WasmEdge_Value *rets, uint32_t rlen, uint8_t *st,
                        uint64_t *cnt);
WasmEdge_Result gather_u64(WasmEdge_BatchContext *C, uint64_t *out,
                           WasmEdge_Result (*f)(WasmEdge_BatchContext *, uint64_t *));
// every shard (stops at the first failure)
template <class F>
WasmEdge_Result all(WasmEdge_BatchContext *C, F f) {
  for (WasmEdge_BatchContext *s : C->shards) {
    if (!s) continue;
    const WasmEdge_Result r = f(s);
    if (r.Code) {
      C->last_error = s->last_error;
      return r;
    }
  }
  return wbh::R(0);
}
inline WasmEdge_BatchContext *first(const WasmEdge_BatchContext *C) {
  for (WasmEdge_BatchContext *s : C->shards)
    if (s) return s;
  return nullptr;
}
}  // namespace wbm
