// batch_api.cpp -- implementation of include/wasmedge_batch.h (the drop-in C ABI).
// Owns the lowered Program, device buffers, one HIP stream per context, and the
// per-instance result buffers.  See the header for the reference interfaces mirrored.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "batch_ctx.h"
#include "build/srchash.h"
#include "jit.h"
#include "multi.h"
#include "tc_slots.h"

extern "C" hipError_t wb_launch_exec(const KParams *p, uint32_t blocks, uint32_t threads,
                                     size_t lds_bytes, int vframe, hipStream_t s);
extern "C" hipError_t wb_launch_wave_order(const uint32_t *ticks, uint32_t *order, uint32_t nwaves,
                                           uint32_t *wave_ctr, hipStream_t s);
extern "C" uint32_t wb_exec_capacity(int vframe, int hbm, int paged, uint32_t threads, size_t lds_bytes);
extern "C" hipError_t wb_launch_mem_init(uint32_t *mem, const uint32_t *image,
                                         uint32_t image_words, uint32_t init_words,
                                         uint32_t mem_words, uint32_t nwaves,
                                         uint32_t *ls, uint32_t ls_slots, uint32_t full,
                                         uint32_t g, uint32_t fuse_state, const uint32_t *global_init,
                                         uint32_t init_pages, uint32_t init_dropped,
                                         uint64_t init_cost, hipStream_t s);
extern "C" hipError_t wb_launch_mem_hash(uint32_t *mem, const uint32_t *ls,
                                         uint32_t ls_slots, uint64_t *hashes,
                                         uint32_t mem_words, uint32_t n, uint32_t g,
                                         const uint64_t *ptab, uint32_t ptab_w, uint32_t max_pages,
                                         hipStream_t s);
extern "C" hipError_t wb_launch_state_init(uint32_t *ls, uint32_t ls_slots, uint32_t nwaves,
                                           const uint32_t *global_init, uint32_t init_pages,
                                           uint32_t init_dropped, uint64_t init_cost, hipStream_t s);


using namespace wbh;

namespace {

// The compiled runs of a V-frame context (jit.h) at the context's current layout
// (C->mlog): assembled, loaded, patched into the threaded code `tcv` and flagged in
// `codepad`. A compile failure is not fatal (the core interprets) but is kept as the last
// error.
void compile_runs(WasmEdge_BatchContext *C, std::vector<DInstr> &codepad, std::vector<TInstr> &tcv) {
  const wb::Program &P = C->prog;
  const bool want_simt = C->want_simt;
  bool want_trip = C->want_trip;
  std::vector<wb::JitRun> runs = wb::jit_runs(P, tcv, want_simt, want_trip);
  if (want_trip && runs.size() > wb::kTripMaxRuns) {   // (too many runs to visit per trip)
    want_trip = false;
    runs = wb::jit_runs(P, tcv, want_simt, false);
  }
  // debugging aids (tools/trip_debug.py): WB_TRIP_LIST=<file> writes the runs' start pcs,
  // WB_TRIP_EXCL=<pc>,<pc>,... leaves the runs starting there to the handlers
  if (const char *tl = getenv("WB_TRIP_LIST"))
    if (FILE *f = fopen(tl, "w")) {
      for (const auto &r : runs) fprintf(f, "%u %u\n", r.pc, r.len);
      fclose(f);
    }
  if (const char *tx = getenv("WB_TRIP_EXCL")) {
    std::vector<uint32_t> ex;
    for (const char *q = tx; *q;) {
      ex.push_back(uint32_t(strtoul(q, const_cast<char **>(&q), 10)));
      if (*q == ',') q++;
      else break;
    }
    runs.erase(std::remove_if(runs.begin(), runs.end(),
                              [&](const wb::JitRun &r) { return std::find(ex.begin(), ex.end(), r.pc) != ex.end(); }),
               runs.end());
  }
  if (!runs.empty()) {
    std::vector<uint8_t> start(P.code.size() + 1, 0);
    for (const auto &r : runs) start[r.pc] = 1;
    std::vector<TInstr> tcj = wb::build_threaded(P, codepad, true, &start, &C->xinfo_h, C->xlog);
    std::vector<uint64_t> addr;
    const wb::JitCost jc{&C->cost_off_h, &C->cost_pool_h, C->cost_else};
    const std::string src = wb::jit_source(P, runs, C->mlog, C->conf.CostLimit ? &jc : nullptr, want_simt,
                                           want_trip, &C->xinfo_h, C->xlog, C->mem_max_pages);
    const std::string err = src.empty() ? std::string("compiled runs: no source")
                                        : wb::jit_load(src, runs.size(), C->device, &addr);
    if (err.empty()) {
      if (C->conf.CostLimit)   // metered: the core holds the runs and nothing else
        for (size_t pc = 0; pc < P.code.size(); pc++) {
          tcj[pc].w[0] = 0;
          codepad[pc].w0 &= ~DBC_HOT;
        }
      wb::jit_patch(tcj, runs, addr);
      for (const auto &r : runs) codepad[r.pc].w0 |= DBC_HOT;   // the core is entered there
      tcv.swap(tcj);
      C->jit_runs = uint32_t(runs.size());
      C->simt = want_simt;
      C->trip = want_trip;
    } else {
      C->last_error = err;
    }
  }
}

uint8_t setup(WasmEdge_BatchContext *C, const uint8_t *wasm, uint32_t len) {
  uint8_t ec = 0;
  std::string err = wb::load_program(wasm, len, C->prog, &ec, C->conf.CostLimit != 0, &C->imports,
                                     C->conf.TailCall != 0, C->conf.MultiMemories != 0);
  if (!err.empty()) return C->fail(ec ? ec : kRuntimeError, err);
  const wb::Program &P = C->prog;
  // gas tables (statistics.h:32: unit costs unless the caller set a table)
  if (C->conf.CostLimit) {
    std::vector<uint64_t> tab(65536, C->conf.CostTable || C->conf.CostTableLen ? 0ull : 1ull);
    for (uint32_t k = 0; C->conf.CostTable && k < C->conf.CostTableLen && k < 65536; k++)
      tab[k] = C->conf.CostTable[k];
    C->init_cost = wb::build_cost_pool(P, tab.data(), C->conf.CostLimit, C->cost_off_h,
                                       C->cost_pool_h, &C->init_exceeded);
    C->cost_else = tab[0x05];
  }
  C->conf.CostTable = nullptr;   // copied: the caller's array need not outlive BatchCreate
  // MemoryInstance(MType, PageLimit) allocates nothing when the initial size exceeds the
  // page limit (include/runtime/instance/memory.h:46-51, test/memlimit/MemLimitTest.cpp:16-18);
  // such an instance is unusable, so the batch fails here instead of running without memory
  if (P.has_mem && C->conf.MaxMemoryPage && P.mem_min > C->conf.MaxMemoryPage)
    return C->fail(kMemoryOutOfBounds, "initial memory pages exceed MaxMemoryPage");
  if (C->conf.DeviceOrdinal >= 0) {
    if (!C->hip_ok(hipSetDevice(C->conf.DeviceOrdinal), "hipSetDevice")) return kRuntimeError;
  }
  (void)hipGetDevice(&C->device);
  if (!C->hip_ok(hipStreamCreateWithFlags(&C->stream, hipStreamNonBlocking), "stream"))
    return kRuntimeError;
  if (!C->hip_ok(hipStreamCreateWithFlags(&C->ctl_stream, hipStreamNonBlocking), "stream"))
    return kRuntimeError;
  if (hipExtMallocWithFlags(reinterpret_cast<void **>(&C->stop), 4, hipDeviceMallocUncached) != hipSuccess &&
      !C->hip_ok(hipMalloc(&C->stop, 4), "interrupt flag"))
    return kRuntimeError;
  (void)hipMemset(C->stop, 0, 4);
  // a lane parked for the host (KParams::parked): a host-mapped word, so a Run with no
  // parked lane skips the service round's status copy (262 KB at 256K instances)
  if (hipHostMalloc(reinterpret_cast<void **>(&C->parked_h), 4, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void **>(&C->parked_d), C->parked_h, 0) != hipSuccess) {
    (void)hipGetLastError();
    if (C->parked_h) (void)hipHostFree(C->parked_h);
    C->parked_h = C->parked_d = nullptr;   // (then every Run takes the service round)
  }
  (void)hipEventCreate(&C->ev0);
  (void)hipEventCreate(&C->ev1);
  hipStream_t s = C->stream;
  C->nwaves = (C->n + 63) / 64;
  // page limit (memory.h:88-115 growPage: 65536, the module's max, PageLimit = MaxMemPage,
  // configure.h:123) and the reserved layout (DESIGN.md "Linear memory"): a module that
  // never grows reserves its initial pages; one that does, more of its limit while the
  // batch's reservation stays small, the rest committed on demand from the pool
  uint32_t limit = 65536;
  if (P.mem_has_max) limit = std::min(limit, P.mem_max);
  if (C->conf.MaxMemoryPage) limit = std::min(limit, C->conf.MaxMemoryPage);
  const bool grows = std::any_of(P.code.begin(), P.code.end(),
                                 [](const DInstr &d) { return (d.w0 & 0x7FFFu) == OP_MEM_GROW; });
  uint32_t reserve = P.mem_min;
  if (grows && limit > P.mem_min) {
    if (C->conf.MemoryReservePages) {
      reserve = std::min(limit, std::max(P.mem_min, C->conf.MemoryReservePages));
    } else {
      size_t free_b = 0, total_b = 0;
      (void)hipMemGetInfo(&free_b, &total_b);
      const uint64_t budget = std::min<uint64_t>(uint64_t(16) << 30, free_b / 4);
      const uint64_t per_lane = budget / (uint64_t(C->nwaves) * (uint64_t(64) << 16));
      reserve = uint32_t(std::max<uint64_t>(P.mem_min, std::min<uint64_t>(limit, per_lane)));
    }
  }
  if (!P.has_mem) reserve = limit = 0;
  C->mem_max_pages = limit;
  C->rpages = C->rpages0 = reserve;
  C->mem_words = reserve << 14;
  C->grow_host = grows && limit > reserve;
  C->pt_n.assign(C->nwaves, 0);
  // interleave granule of the wave's linear memories (DESIGN.md "Linear memory"): 4-byte
  // words when the module's addresses are wave-uniform, wider granules (a lane's
  // consecutive words together) when they diverge per lane (Program::divergent_mem)
  uint32_t gb = C->conf.MemoryGranule;
  if (const char *e = getenv("WB_GRANULE")) gb = uint32_t(atoi(e));
  // a module whose addresses may differ between instances starts at 128-byte granules and
  // tries 4-byte words on its second run (layout_trial; WB_GRANULE_TRIAL=0 turns it off)
  const char *gte = getenv("WB_GRANULE_TRIAL");
  if (gb == 0 && P.divergent_mem && P.has_mem && !(gte && gte[0] == '0')) {
    C->trial = 5;   // (the first run warms up unmeasured: a cold run would favour a switch)
    C->trial_mlog[0] = 5;   // 128 B
    C->trial_mlog[1] = 0;   // 4 B
  }
  if (gb == 0) gb = P.divergent_mem ? 128 : 4;   // profiles/r02h_c3_granules.json
  if (gb < 4 || gb > 128 || (gb & (gb - 1)))
    return C->fail(kRuntimeError, "MemoryGranule must be 0 or a power of two in [4, 128]");
  C->mlog = uint32_t(__builtin_ctz(gb)) - 2;
  // the call stack: a fixed CallStackCells, or (0) 4096 cells that grow on demand
  // (WB_STACK_GROW=0 keeps them fixed: A/B and test aid)
  C->gs_depth = C->conf.CallStackCells ? C->conf.CallStackCells : 4096;
  const char *sge = getenv("WB_STACK_GROW");
  C->gs_grow = !C->conf.CallStackCells && !(sge && sge[0] == '0');
  C->gs_grow0 = C->gs_grow;
  C->gs_depth0 = C->gs_depth;
  // per-lane tables widen past their first capacity up to table_widen_limit (WB_TABLE_WIDEN=0
  // keeps the first capacity: test aid)
  std::vector<uint32_t> tlim;
  const char *twe = getenv("WB_TABLE_WIDEN");
  if (P.mut_tables && !(twe && twe[0] == '0'))
    for (uint32_t t = 0; t < P.ntables; t++) {
      tlim.push_back(wb::table_widen_limit(P.tables[t]));
      C->tg_grow |= tlim.back() > P.tabinfo[2 * t + 1];
    }
  if (!C->tg_grow) tlim.clear();
  // module image: active data segments over the initial pages
  std::vector<uint32_t> img;
  std::vector<uint8_t> pool;
  std::vector<uint32_t> doff, dlen;
  std::vector<uint32_t> dropped((P.datas.size() + 31) / 32 + 1, 0u);   // a bit per data segment
  for (size_t k = 0; k < P.datas.size(); k++) {
    const auto &d = P.datas[k];
    doff.push_back(uint32_t(pool.size()));
    dlen.push_back(uint32_t(d.bytes.size()));
    pool.insert(pool.end(), d.bytes.begin(), d.bytes.end());
    if (d.active) dropped[k >> 5] |= 1u << (k & 31);   // active segments are dropped after init
    if (d.active && !d.mem) {   // (memory 0's image; the others' below)
      uint64_t end = uint64_t(d.offset) + d.bytes.size();
      if (img.size() * 4 < end) img.resize((end + 3) / 4, 0);
      for (size_t b = 0; b < d.bytes.size(); b++) {
        uint32_t a = d.offset + uint32_t(b);
        img[a >> 2] = (img[a >> 2] & ~(0xFFu << (8 * (a & 3)))) | (uint32_t(d.bytes[b]) << (8 * (a & 3)));
      }
    }
  }
  C->image_words = uint32_t(img.size());
  C->init_dropped = dropped[0];
  // memories past the first (MultiMemories): every lane's are reserved whole -- the
  // initial size, or with a memory.grow on it up to its page limit as far as a budget of
  // min(4 GiB, an eighth of the free device memory) goes -- back to back, in 4-byte words
  // interleaved over a wave's lanes; only the per-lane step addresses them (KParams::xmem).
  // A grow past the reservation returns -1 (the allocation failing, allocator.cpp:101-129).
  std::vector<uint32_t> ximg;
  if (!P.xmems.empty()) {
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    const uint64_t budget = std::min<uint64_t>(uint64_t(4) << 30, free_b / 8);
    const uint64_t per_lane = budget / (uint64_t(C->nwaves) * 64 * 65536 * P.xmems.size());
    uint64_t words = 0;
    for (size_t k = 0; k < P.xmems.size(); k++) {
      const auto &xm = P.xmems[k];
      uint32_t lim = xm.has_max ? std::min<uint32_t>(xm.max, 65536) : 65536;
      if (C->conf.MaxMemoryPage) lim = std::min(lim, C->conf.MaxMemoryPage);
      if (xm.min > lim) return C->fail(kMemoryOutOfBounds, "initial memory pages exceed MaxMemoryPage");
      bool grows = false;
      for (const auto &I : P.code)
        grows |= (I.w0 & 0xFFFFu) == OP_XMEM_GROW && (I.w1 >> 16) == k + 1;
      const uint64_t want = C->conf.ExtraMemoryReservePages ? C->conf.ExtraMemoryReservePages : per_lane;
      const uint32_t res = grows ? uint32_t(std::max<uint64_t>(xm.min, std::min<uint64_t>(lim, want))) : xm.min;
      C->xinfo_h.push_back(uint32_t(words));
      C->xinfo_h.push_back(res);
      words += uint64_t(res) << 14;
      if (words > 0xFFFFFFFFull) return C->fail(kRuntimeError, "memories past the first exceed 16 GiB per instance");
    }
    C->xwords = uint32_t(words);
    // their granule, fixed here (no layout trial: memory 0's picks its own): 128 bytes when
    // some access to them depends on per-instance data (Program::divergent_xmem: a lane's
    // nearby words then share a cache line, as memory 0's default), else 4 (lanes' words
    // side by side, coalesced where they move together). WB_XGRAN=<bytes> forces one (A/B).
    const char *xge = getenv("WB_XGRAN");
    const uint32_t xgb = xge ? uint32_t(atoi(xge)) : P.divergent_xmem ? 128u : 4u;
    C->xlog = 0;
    while (C->xlog < 5 && (4u << C->xlog) < xgb) C->xlog++;
    ximg.assign(C->xwords, 0u);
    for (const auto &d : P.datas) {
      if (!d.active || !d.mem) continue;
      const uint64_t b0 = uint64_t(C->xinfo_h[2 * (d.mem - 1)]) * 4 + d.offset;
      for (size_t b = 0; b < d.bytes.size(); b++) {
        const uint64_t a = b0 + b;
        ximg[a >> 2] = (ximg[a >> 2] & ~(0xFFu << (8 * (a & 3)))) | (uint32_t(d.bytes[b]) << (8 * (a & 3)));
      }
    }
    C->xpages0.assign(P.xmems.size() * size_t(C->nwaves) * 64, 0u);
    for (size_t k = 0; k < P.xmems.size(); k++)
      std::fill(C->xpages0.begin() + k * size_t(C->nwaves) * 64, C->xpages0.begin() + (k + 1) * size_t(C->nwaves) * 64,
                P.xmems[k].min);
  }
  std::vector<DFunc> fv;
  for (const auto &f : P.funcs)
    fv.push_back(DFunc{f.imported ? 0xFFFFFFFFu : f.entry_pc, P.type_canon[f.type]});
  std::vector<DInstr> codepad = P.code;   // +1: the kernel prefetches pc+1
  codepad.push_back(DInstr{0, 0, 0, 0});
  // threaded code for the hand-written dispatch core; WB_THREADED=0 runs every op
  // through the compiled step instead (A/B measurement aid)
  const char *thr = getenv("WB_THREADED");
  C->threaded = !(thr && thr[0] == '0');
  // frames that LDS cannot hold (a 64-lane cell row is 256 B; ~640 cells per wave at one
  // wave per block) live in HBM and run in the compiled step; WB_HBMFRAME=1 forces it
  // (A/B and test aid)
  const char *hfe = getenv("WB_HBMFRAME");
  C->frame_hbm = (size_t(P.total_cells()) + 1) * 256 + 256 > 150 * 1024 || (hfe && hfe[0] == '1');
  if (C->frame_hbm) C->threaded = false;
  std::vector<TInstr> tcv;
  // V frames (frame cells in VGPRs while the core runs) when the frame fits in
  // v128..v255: 2 waves per SIMD (256 VGPRs), against 4 for the LDS kernel, but the
  // compiled runs and SIMT scheduling only exist for V frames (C5 at 256K instances =
  // 4 waves per SIMD: 1.60e12 instr/s against 1.13e12). WB_VFRAME=0 / 1 forces LDS / V
  // frames (A/B measurement aid).
  const char *vfe = getenv("WB_VFRAME");
  const char *sce = getenv("WB_SCHED");
  C->sched = sce ? (uint32_t)atoi(sce) : 1u;
  // modules without a scan loop keep plain min-pc scheduling (no loop-table lookups)
  if (std::all_of(P.loops.begin(), P.loops.end(), [](uint32_t v) { return v == 0xFFFFFFFFu; }))
    C->sched = 0;
  const bool vf_fit = C->threaded && P.total_cells() <= TC_VF_CELLS;
  C->vframe = vf_fit && (vfe ? vfe[0] == '1' : true);
  if (C->threaded) tcv = wb::build_threaded(P, codepad, C->vframe, nullptr, &C->xinfo_h, C->xlog);
  // compiled runs (jit.h) for the V-frame core; WB_JIT=0 interprets them instead. A
  // compile failure is not fatal (the core interprets) but is kept as the last error.
  const char *jte = getenv("WB_JIT");
  // Metered contexts run only the compiled runs in the core (they price themselves,
  // JitCost); every other instruction stays in the exact compiled / per-lane step.
  // SIMT scheduling inside the compiled runs (KParams::simt), not for metered contexts;
  // WB_SIMT=0 turns it off (A/B measurement aid). (C3 4K: 1.19e11 instr/s against 9.8e10
  // with the kernel's scan-loop policy between core calls.)
  const char *sme = getenv("WB_SIMT");
  const bool want_simt = !C->conf.CostLimit && !(sme && sme[0] == '0');
  // Trip mode (jit.h) for modules whose load/store addresses depend on per-instance data
  // (Program::divergent_mem: lanes part ways on loaded data) and for call-free modules
  // whose lanes part ways inside their loops (wb::trips_pay); WB_TRIP=0 / 1 forces it off /
  // on (A/B measurement aid). SIMT contexts only.
  const char *tre = getenv("WB_TRIP");
  bool want_trip = want_simt && (tre ? tre[0] == '1' : P.divergent_mem || P.divergent_xmem || wb::trips_pay(P));
  C->want_simt = want_simt;
  C->want_trip = want_trip;
  C->jit_on = C->threaded && C->vframe && !(jte && jte[0] == '0');
  C->codepad0 = codepad;   // (pristine: a change of layout compiles the runs again)
  if (C->jit_on) compile_runs(C, codepad, tcv);
  // LS image from slot LS_GLOBALS on: globals, then (per-lane tables) table sizes and
  // the dropped-elem mask
  std::vector<uint32_t> ls_init = P.global_init;
  if (P.mut_tables) {
    for (const auto &t : P.tables) ls_init.push_back(t.min);
    ls_init.insert(ls_init.end(), P.init_edropped.begin(), P.init_edropped.end());
  }
  // the dropped-data mask past its first word (data segments 32 on)
  C->ls_drop_ext = LS_GLOBALS + uint32_t(ls_init.size());
  ls_init.insert(ls_init.end(), dropped.begin() + 1, dropped.end());
  bool ok = C->code.upload(codepad, s) && C->loops.upload(P.loops, s) && (!C->threaded || C->tcode.upload(tcv, s)) && C->brtab.upload(P.brtab, s) &&
            C->vconst.upload(P.vconst, s) && C->table.upload(P.table0, s) &&
            C->global_init.upload(ls_init, s) && C->image.upload(img, s) &&
            C->tab_image.upload(P.tab_image, s) && C->tabinfo.upload(P.tabinfo, s) &&
            C->elem_pool.upload(P.elem_pool, s) && C->elem_off.upload(P.elem_off, s) &&
            C->elem_len.upload(P.elem_len, s) && (!C->tg_grow || C->tlimit.upload(tlim, s)) &&
            (!C->conf.CostLimit || (C->cost_off.upload(C->cost_off_h, s) &&
                                    C->cost_pool.upload(C->cost_pool_h, s))) &&
            C->funcs.upload(fv, s) && C->data_pool.upload(pool, s) &&
            C->data_off.upload(doff, s) && C->data_len.upload(dlen, s) &&
            (P.xmems.empty() || (C->ximage.upload(ximg, s) && C->xinfo.upload(C->xinfo_h, s)));
  if (!ok) return C->fail(kRuntimeError, "device allocation/upload of the module failed");
  size_t nw = C->nwaves;
  C->ls_slots = LS_GLOBALS + uint32_t(ls_init.size());
  // LDS call-stack slots per lane: what the frames leave of the LDS share each wave gets
  // at the occupancy this batch reaches (nwaves over 256 CUs, at most 16 waves per CU)
  {
    const uint32_t tc = C->frame_hbm ? 0 : P.total_cells() ? P.total_cells() : 1;
    const uint32_t lw = C->nwaves;   // launch waves
    const uint32_t per_cu = std::min<uint32_t>(C->vframe ? 8 : 16, std::max<uint32_t>(4, (lw + 255) / 256));
    const uint32_t wave_cells = (160 * 1024 - 1024) / 256 / per_cu;   // 256 B per cell row
    uint32_t s = wave_cells > tc + 1 ? wave_cells - tc - 1 : 0;
    if (s > C->gs_depth) s = C->gs_depth;
    C->gs_lds = s >= 8 ? s : 0;
  }
  C->hosts.assign(P.funcs.size(), {});
  C->hb_cells = 1;
  for (uint32_t f = 0; f < P.n_imported; f++) {
    uint32_t a = 0, r = 0;
    for (uint8_t t : P.types[P.funcs[f].type].params) a += wb::cells_of(t);
    for (uint8_t t : P.types[P.funcs[f].type].results) r += wb::cells_of(t);
    C->hb_cells = std::max(C->hb_cells, std::max(a, r));
  }
  if (!C->mem.alloc(nw * size_t(C->mem_words) * 64 + 64) ||
      !C->gstack.alloc(nw * size_t(C->gs_depth) * 64) ||
      !C->lstate.alloc(nw * size_t(C->ls_slots) * 64) || !C->status.alloc(C->n + 1) ||
      !C->ltab.alloc(nw * size_t(P.tab_words) * 64) ||
      !C->counts.alloc(C->n + 1) || !C->hashes.alloc(C->n + 1) ||
      (!P.xmems.empty() && (!C->xmem.alloc(nw * 64 * size_t(C->xwords) + 64) ||
                            !C->xpages.alloc(C->xpages0.size()))) ||
      (C->frame_hbm && !C->hframe.alloc(nw * size_t(P.total_cells()) * 64)) ||
      ((P.n_imported || C->grow_host || C->gs_grow || C->tg_grow) && (!C->fsave.alloc(nw * size_t(P.total_cells() + C->gs_lds) * 64) ||
                        !C->hcall.alloc(C->n) || !C->hbuf.alloc(size_t(C->n) * C->hb_cells))))
    return C->fail(kRuntimeError, "device allocation of instance state failed (" +
                                      std::to_string(nw * size_t(C->mem_words) * 256 >> 20) +
                                      " MiB linear memory)");
#ifdef WB_STATS
  if (!C->hip_ok(hipMalloc(&C->stats, (nw * 32 + 1024) * sizeof(uint64_t)), "stats")) return kRuntimeError;
#endif
  if (!C->hip_ok(hipStreamSynchronize(s), "upload")) return kRuntimeError;
  return 0;
}

// A new interleave granule (at a Reset, which then writes every page of every lane): the
// compiled runs again at the new layout.
uint8_t relayout(WasmEdge_BatchContext *C, uint32_t mlog) {
  if (!C->settle()) return kRuntimeError;
  C->mlog = mlog;
  if (C->jit_on) {
    std::vector<DInstr> codepad = C->codepad0;
    std::vector<TInstr> tcv = wb::build_threaded(C->prog, codepad, C->vframe);
    C->jit_runs = 0;
    C->simt = C->trip = false;
    compile_runs(C, codepad, tcv);
    if (!C->code.upload(codepad, C->stream) || !C->tcode.upload(tcv, C->stream))
      return C->fail(kRuntimeError, "device upload of the module failed");
  }
  C->mem_fresh = true;
  return 0;
}

// Layout trial: the interleave granule from observed throughput, for modules whose
// addresses may differ between instances (Program::divergent_mem; the static analysis
// cannot tell a per-lane index from a wave-uniform one kept in memory, such as mt19937's
// state index). After one unmeasured warm-up run, a run at 128-byte granules and the next
// one, after a Reset, at 4-byte words each measure wasm instructions per kernel second; the
// 4-byte layout stays when it is at least 10% faster on the same function, else the next
// Reset goes back. The rate is per instruction, so runs on different arguments compare.
// Trial runs do not use the longest-first wave order, so both see the same schedule.
// Results never depend on the layout (tests/test_workloads.py granule matrix).
uint8_t layout_trial(WasmEdge_BatchContext *C, double secs) {
  std::vector<uint64_t> cnt(C->n);
  if (secs <= 0 || !C->hip_ok(hipMemcpy(cnt.data(), C->counts.ptr, size_t(C->n) * 8, hipMemcpyDeviceToHost), "counts")) {
    C->trial = C->trial == 3 ? 4 : 0;
    return secs <= 0 ? 0 : kRuntimeError;
  }
  double sum = 0;
  for (uint64_t c : cnt) sum += double(c);
  const double rate = sum / secs;
  if (C->trial == 1) {
    C->trial_rate = rate;
    C->trial_func = C->func;
    C->trial = 2;
  } else {   // 3
    C->trial = C->func == C->trial_func && rate >= 1.10 * C->trial_rate ? 0 : 4;
  }
  return 0;
}

uint32_t cells_of_value(uint8_t t) { return wb::cells_of(t); }

// One interpreter launch over every instance: entry_pc with the staged params (or the
// start function when is_start). Shared by BatchRun and BatchReset.
uint8_t launch_once(WasmEdge_BatchContext *C, uint32_t entry_pc, bool is_start, bool resume,
                    double *KernelSeconds) {
  const wb::Program &P = C->prog;
  KParams k{};
  k.code = C->code.ptr; k.brtab = C->brtab.ptr; k.vconst = C->vconst.ptr;
  k.funcs = C->funcs.ptr; k.table = C->table.ptr; k.global_init = C->global_init.ptr;
  k.data_pool = C->data_pool.ptr; k.data_off = C->data_off.ptr; k.data_len = C->data_len.ptr;
  // metered runs take the exact compiled step (the threaded core counts per run only)
  k.tcode = C->threaded && (!C->conf.CostLimit || C->jit_runs) ? C->tcode.ptr : nullptr;
  // gas: the instance's running total against the limit, start function included
  k.cost_limit = C->conf.CostLimit ? C->conf.CostLimit : ~0ull;
  if (C->conf.CostLimit) {
    k.cost_off = C->cost_off.ptr;
    k.cost_pool = C->cost_pool.ptr;
    k.cost_else = C->cost_else;
  }
  k.stop = C->stop;
  if (P.mut_tables) {
    k.ltab = C->ltab.ptr; k.tabinfo = C->tabinfo.ptr; k.elem_pool = C->elem_pool.ptr;
    k.elem_off = C->elem_off.ptr; k.elem_len = C->elem_len.ptr;
    k.mut_tables = 1; k.ntables = P.ntables; k.tab_words = P.tab_words;
  }
  k.ls_tab = LS_GLOBALS + P.global_cells;
  k.ls_drop_ext = C->ls_drop_ext;
  k.mem = C->mem.ptr; k.gstack = C->gstack.ptr; k.lstate = C->lstate.ptr;
  k.fsave = C->fsave.ptr; k.hcall = C->hcall.ptr; k.hbuf = C->hbuf.ptr;
  k.hframe = C->frame_hbm ? C->hframe.ptr : nullptr;
  k.params = is_start ? nullptr : C->params.ptr;
  k.results = is_start ? nullptr : C->results.ptr;
  k.status = C->status.ptr; k.counts = C->counts.ptr;
  k.n = C->n;
  k.entry_pc = entry_pc;
  k.param_cells = is_start ? 0 : C->param_cells;
  k.result_cells = is_start ? 0 : C->result_cells;
  k.global_cells = P.global_cells;
  k.total_cells = P.total_cells() ? P.total_cells() : 1;
  k.table_size = uint32_t(P.table0.size());
  k.mem_words = C->mem_words;
  k.mlog = C->mlog;
  k.init_pages = P.mem_min;
  k.mem_max_pages = C->mem_max_pages;
  k.rpages = C->rpages;
  k.ptab = C->pt_w ? C->ptab.ptr : nullptr;
  k.ptab_w = C->pt_w;
  k.grow_host = C->grow_host ? 1u : 0u;
  k.gs_depth = C->gs_depth;
  k.gs_lds = C->gs_lds;
  k.gs_grow = C->gs_grow ? 1u : 0u;
  k.tg_grow = C->tg_grow ? 1u : 0u;
  k.tlimit = C->tlimit.ptr;
  k.parked = C->parked_d;
  if (!P.xmems.empty()) {
    k.xmem = C->xmem.ptr; k.xpages = C->xpages.ptr; k.xinfo = C->xinfo.ptr;
    k.xwords = C->xwords; k.xstride = C->nwaves * 64; k.n_xmem = uint32_t(P.xmems.size());
    k.xlog = C->xlog;
  }
  k.init_dropped = C->init_dropped;
  k.ls_slots = C->ls_slots;
  k.is_start = is_start ? 1u : 0u;
  k.resume = resume ? 1u : 0u;
  k.hb_cells = C->hb_cells;
  k.max_steps = C->conf.MaxSteps ? C->conf.MaxSteps : (1ull << 62);
  double tl = C->conf.TimeLimitSeconds > 0 ? C->conf.TimeLimitSeconds : 600.0;
  k.max_ticks = uint64_t(tl * 1e8);
  k.sched = C->sched;
  k.loops = C->loops.ptr;
  k.simt = C->simt && k.tcode ? 1u : 0u;
  k.stats = C->stats;
#ifdef WB_STATS
  (void)hipMemsetAsync(C->stats, 0, (size_t(C->nwaves) * 32 + 1024) * sizeof(uint64_t), C->stream);
#endif
  // launch geometry: 4 waves per block when their LDS frames fit in 160 KB
  size_t wave_lds = size_t((C->frame_hbm ? 0 : k.total_cells) + k.gs_lds) * 64 * 4;
  if (wave_lds + 256 > 160 * 1024)
    return C->fail(kRuntimeError, "internal: LDS share of a wave exceeds 160 KiB");
  uint32_t wpb = 4;
  while (wpb > 1 && wave_lds * wpb + 256 > 160 * 1024) wpb >>= 1;
  uint32_t blocks = (C->nwaves + wpb - 1) / wpb;
  // persistent waves when the batch has more waves than the device holds at once (C5: 4,096
  // waves, 2 per SIMD): as many blocks as fit, each wave taking the next batch wave when
  // its own ends (batch_kernel.hip next_wave); WB_PERSIST=0 launches a wave per batch wave
  const bool vf = C->vframe && k.tcode;
  if (C->cap_threads != wpb * 64 || C->cap_lds != wave_lds * wpb + 256) {
    C->cap_threads = wpb * 64;
    C->cap_lds = wave_lds * wpb + 256;
    C->cap_blocks = wb_exec_capacity(vf, k.hframe != nullptr, k.grow_host || k.n_xmem, C->cap_threads, C->cap_lds);
  }
  const char *pe = getenv("WB_PERSIST");
  if (const char *lp = getenv("WB_LPT")) C->lpt = lp[0] != '0';
  if (C->cap_blocks && blocks > C->cap_blocks && !(pe && pe[0] == '0')) {
    if (!C->wave_ctr.ptr && !C->wave_ctr.alloc(1)) return C->fail(kRuntimeError, "device allocation failed");
    // the last launch's wave-order kernel (its own stream): it zeroed the counter, and wrote
    // the order this launch reads from the ticks this launch overwrites
    if (C->order_pending && !C->hip_ok(hipStreamWaitEvent(C->stream, C->ev_order, 0), "wave order wait"))
      return kRuntimeError;
    C->order_pending = false;
    // (the wave-order kernel after the last launch zeroed it already)
    if (!C->ctr_zero && !C->hip_ok(hipMemsetAsync(C->wave_ctr.ptr, 0, 4, C->stream), "wave counter"))
      return kRuntimeError;
    C->ctr_zero = false;
    k.wave_ctr = C->wave_ctr.ptr;
    blocks = C->cap_blocks;
    // longest-first order from the last launch of this function (batch_ctx.h wave_order)
    if (C->lpt && !resume && !is_start) {
      if (!C->wave_ticks.ptr && (!C->wave_ticks.alloc(C->nwaves) || !C->wave_order.alloc(C->nwaves)))
        return C->fail(kRuntimeError, "device allocation failed");
      k.wave_ticks = C->wave_ticks.ptr;
      // (only for the same function on the same arguments: waves of other inputs take
      // other times, and an order learned from them is noise -- the fresh-input bench)
      // (WB_ORDER_ANY=1: also on other arguments -- an experiment, the per-slot cost of the
      // last launch as the guess)
      const char *oae = getenv("WB_ORDER_ANY");
      const bool any_args = oae && oae[0] == '1';
      k.wave_order = C->order_pc == entry_pc && (C->order_fp == C->args_fp || any_args) && C->trial != 1 &&
                             C->trial != 3
                         ? C->wave_order.ptr : nullptr;
    }
  }
  // a Reset left to this launch (WasmEdge_BatchReset): each wave does its part first
  const bool rf = C->reset_deferred && !resume && !is_start;
  if (rf) {
    k.rf_on = 1;
    k.rf_image = C->image.ptr;
    k.rf_image_words = C->image_words;
    k.rf_init_words = C->mem_words;
    k.rf_global_init = C->global_init.ptr;
    k.rf_init_pages = P.mem_min;
    k.rf_init_dropped = C->init_dropped;
    k.rf_init_cost = C->init_cost;
  } else if (C->reset_deferred && !wbh_reset_now(C)) {
    return kRuntimeError;
  }
  (void)hipEventRecord(C->ev0, C->stream);
  // +1 cell row: the threaded core reads operand cells k and k+1 (ds_read2_b32)
  if (!C->hip_ok(wb_launch_exec(&k, blocks, wpb * 64, wave_lds * wpb + 256, vf, C->stream), "launch"))
    return kRuntimeError;
  if (rf) C->reset_deferred = false;
  (void)hipEventRecord(C->ev1, C->stream);
  // the next launch of this function takes the longest waves first (sorted on the device,
  // after the timed kernel, on a stream of its own so that it overlaps the next Reset; the
  // order buffer is only read by later launches)
  if (k.wave_ticks) {
    if (!C->order_stream &&
        (!C->hip_ok(hipStreamCreateWithFlags(&C->order_stream, hipStreamNonBlocking), "stream") ||
         !C->hip_ok(hipEventCreateWithFlags(&C->ev_order, hipEventDisableTiming), "event")))
      return kRuntimeError;
    if (!C->hip_ok(hipStreamWaitEvent(C->order_stream, C->ev1, 0), "wave order wait") ||
        !C->hip_ok(wb_launch_wave_order(k.wave_ticks, C->wave_order.ptr, C->nwaves, C->wave_ctr.ptr,
                                        C->order_stream), "wave order") ||
        !C->hip_ok(hipEventRecord(C->ev_order, C->order_stream), "wave order"))
      return kRuntimeError;
    C->order_pending = true;
    C->order_pc = entry_pc;
    C->order_fp = C->args_fp;
    C->ctr_zero = true;
  }
  // the interpreter kernel's end
  if (!C->hip_ok(hipEventSynchronize(C->ev1), "interpreter kernel")) return kRuntimeError;
  C->reset_pending = false;   // (the instance state is final)
  if (KernelSeconds) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, C->ev0, C->ev1);
    *KernelSeconds += ms * 1e-3;
  }
  return 0;
}

// One interpreter invocation over every instance: entry_pc with the staged params (or the
// start function when is_start), then host-import rounds until no lane is parked.
// Shared by BatchRun and BatchReset.
uint8_t launch_exec(WasmEdge_BatchContext *C, uint32_t entry_pc, bool is_start,
                    double *KernelSeconds) {
  if (KernelSeconds) *KernelSeconds = 0;
  // (the flag is cleared only after an Interrupt: one stream operation less per run)
  if (C->stop_dirty.exchange(false) &&
      !C->hip_ok(hipMemsetAsync(C->stop, 0, 4, C->stream), "interrupt flag")) return kRuntimeError;
  if (C->parked_h) *C->parked_h = 0u;   // (the previous launch has ended: launch_once syncs)
  uint8_t e = launch_once(C, entry_pc, is_start, false, KernelSeconds);
  if (e || !(C->prog.n_imported || C->grow_host || C->gs_grow || C->tg_grow)) return e;
  for (;;) {
    if (C->parked_h && !__atomic_load_n(C->parked_h, __ATOMIC_ACQUIRE)) return 0;   // none parked
    if (C->parked_h) *C->parked_h = 0u;
    // every round resumes the lanes the host serviced; lanes it ended keep its code
    const int64_t k = service_host_calls(C);
    if (k < 0) return kRuntimeError;
    if (k == 0) return 0;
    e = launch_once(C, entry_pc, is_start, true, KernelSeconds);
    if (e) return e;
  }
}

}  // namespace

// (batch_ctx.h) the Reset a launch was to fold in, as wb_mem_init_kernel's write-mark path
bool wbh_reset_now(WasmEdge_BatchContext *C) {
  C->reset_deferred = false;
  const wb::Program &P = C->prog;
  if (!C->hip_ok(wb_launch_mem_init(C->mem.ptr, C->image.ptr, C->image_words, C->mem_words, C->mem_words,
                                    C->nwaves, C->lstate.ptr, C->ls_slots, 0u, C->mlog, 1u,
                                    C->global_init.ptr, P.mem_min, C->init_dropped, C->init_cost,
                                    C->stream), "mem init"))
    return false;
  C->reset_pending = true;
  return true;
}

extern "C" {

WasmEdge_BatchContext *WasmEdge_BatchCreate(const WasmEdge_BatchConfigure *Conf,
                                            const uint8_t *WasmBuf, uint32_t WasmLen,
                                            uint32_t NumInstances, WasmEdge_Result *Res) {
  return WasmEdge_BatchCreateWithImports(Conf, WasmBuf, WasmLen, NumInstances, nullptr, 0, Res);
}

WasmEdge_BatchContext *WasmEdge_BatchCreateWithImports(const WasmEdge_BatchConfigure *Conf,
                                                       const uint8_t *WasmBuf, uint32_t WasmLen,
                                                       uint32_t NumInstances,
                                                       const WasmEdge_BatchImport *Imports,
                                                       uint32_t ImportLen, WasmEdge_Result *Res) {
  if (!WasmBuf || NumInstances == 0) {
    g_last_create_error = "null buffer or zero instances";
    if (Res) *Res = R(kWrongVMWorkflow);
    return nullptr;
  }
  if (Conf && Conf->DeviceCount > 1)   // several devices: a parent over one shard each
    return wbm::create(*Conf, WasmBuf, WasmLen, NumInstances, Imports, ImportLen, Res);
  auto *C = new WasmEdge_BatchContext();
  if (Conf) C->conf = *Conf;
  else C->conf.DeviceOrdinal = -1;
  C->host_threads = C->conf.HostThreads;
  C->n = NumInstances;
  for (uint32_t k = 0; Imports && k < ImportLen; k++) {
    const WasmEdge_BatchImport &I = Imports[k];
    wb::HostImport h;
    h.module.assign(I.ModuleName.Buf ? I.ModuleName.Buf : "", I.ModuleName.Length);
    h.name.assign(I.ExternalName.Buf ? I.ExternalName.Buf : "", I.ExternalName.Length);
    h.kind = uint8_t(I.Kind);
    h.type = uint8_t(I.Type);
    h.mut = I.Mutable != 0;
    h.min = I.Min;
    h.max = I.Max;
    h.has_max = I.HasMax != 0;
    bool full = false;
    const uint128_t iv = I.Kind == WASMEDGE_BATCH_IMPORT_GLOBAL && I.Type == WasmEdge_ValType_ExternRef
                             ? uint128_t(C->xref_in(I.Value.Value, &full)) : I.Value.Value;
    if (full) {
      if (Res) *Res = R(kRuntimeError);
      delete C;
      return nullptr;
    }
    for (uint32_t q = 0; q < 4; q++) h.value[q] = uint32_t(iv >> (32 * q));
    C->imports.push_back(h);
  }
  uint8_t e = setup(C, WasmBuf, WasmLen);
  if (!e) e = WasmEdge_BatchReset(C, nullptr).Code;   // instantiate every instance
  if (e) {
    g_last_create_error = C->last_error;
    if (Res) *Res = R(e);
    WasmEdge_BatchDelete(C);
    return nullptr;
  }
  if (Res) *Res = R(0);
  return C;
}

WasmEdge_Result WasmEdge_BatchSetArgs(WasmEdge_BatchContext *C, const WasmEdge_String FuncName,
                                      const WasmEdge_Value *Params, const uint32_t ParamLen) {
  if (!C) return R(kWrongVMWorkflow);
  if (!C->shards.empty()) return wbm::set_args(C, FuncName, Params, ParamLen);
  DevScope dev(C);
  std::string name(FuncName.Buf ? FuncName.Buf : "", FuncName.Length);
  int f = wb::find_export(C->prog, name);
  if (f < 0) return R(C->fail(kFuncNotFound, "function '" + name + "' not found"));
  const wb::FuncType &t = C->prog.types[C->prog.funcs[f].type];
  // executor.cpp:88-100: parameter count and types must match
  if (ParamLen != t.params.size()) return R(C->fail(kFuncSigMismatch, "parameter count mismatch"));
  uint32_t pc = 0;
  for (uint8_t ty : t.params) pc += cells_of_value(ty);
  std::vector<uint32_t> cells(size_t(C->n) * (pc ? pc : 1));
  for (uint32_t i = 0; i < C->n; i++) {
    uint32_t at = 0;
    for (uint32_t k = 0; k < ParamLen; k++) {
      const WasmEdge_Value &v = Params[size_t(i) * ParamLen + k];
      if (uint8_t(v.Type) != t.params[k])
        return R(C->fail(kFuncSigMismatch, "parameter type mismatch"));
      bool full = false;
      const uint128_t x = t.params[k] == wb::EXTERNREF ? uint128_t(C->xref_in(v.Value, &full)) : v.Value;
      if (full) return R(C->fail(kRuntimeError, "externref intern table full (2^31 - 1 values)"));
      for (uint32_t q = 0; q < cells_of_value(t.params[k]); q++)
        cells[size_t(i) * pc + at++] = uint32_t(x >> (32 * q));
    }
  }
  uint32_t rc = 0;
  for (uint8_t ty : t.results) rc += cells_of_value(ty);
  // (the buffers stay when their sizes do: a caller passing new arguments every run pays no
  // device allocation, and the kernel reads the same pages)
  const size_t rn = size_t(C->n) * (rc ? rc : 1);
  if ((C->params.n != cells.size() || !C->params.ptr) && !C->params.alloc(cells.size()))
    return R(C->fail(kRuntimeError, "device allocation failed"));
  if ((C->results.n != rn || !C->results.ptr) && !C->results.alloc(rn))
    return R(C->fail(kRuntimeError, "device allocation failed"));
  if (!C->hip_ok(hipMemcpyAsync(C->params.ptr, cells.data(), cells.size() * 4,
                                hipMemcpyHostToDevice, C->stream), "params upload"))
    return R(kRuntimeError);
  if (!C->hip_ok(hipStreamSynchronize(C->stream), "params upload")) return R(kRuntimeError);
  // fingerprint of the arguments (the longest-first wave order is reused only on equal ones)
  uint64_t fp = 0x9E3779B97F4A7C15ull ^ uint64_t(f);
  for (uint32_t c : cells) fp = (fp ^ c) * 0x100000001B3ull + (fp >> 29);
  C->args_fp = fp;
  C->func = f;
  C->param_cells = pc;
  C->result_cells = rc;
  C->result_types = t.results;
  return R(0);
}

WasmEdge_Result WasmEdge_BatchReset(WasmEdge_BatchContext *C, double *KernelSeconds) {
  if (!C) return R(kWrongVMWorkflow);
  if (!C->shards.empty()) return wbm::reset(C, KernelSeconds);
  DevScope dev(C);
  const wb::Program &P = C->prog;
  if (C->trial == 2 || C->trial == 4) {   // (layout_trial)
    const uint8_t e = relayout(C, C->trial_mlog[C->trial == 2 ? 1 : 0]);
    if (e) return R(e);
    C->trial = C->trial == 2 ? 3 : 0;
  }
  // lanes grew into pool rows: the layout takes every page they reached (hostcall.cpp
  // grow_layout; this Reset rewrites every page, so nothing is copied)
  if (C->grow_host && C->pool_used) {
    if (!C->settle()) return R(kRuntimeError);
    const size_t row = 64 * sizeof(uint32_t), pitch = size_t(C->ls_slots) * row;
    std::vector<uint32_t> pages(size_t(C->nwaves) * 64);
    if (!C->hip_ok(hipMemcpy2D(pages.data(), row, C->lstate.ptr + LS_PAGES * 64, pitch, row, C->nwaves,
                               hipMemcpyDeviceToHost), "pages"))
      return R(kRuntimeError);
    uint32_t reached = 0;
    for (uint32_t i = 0; i < C->n; i++) reached = std::max(reached, pages[i]);
    if (!grow_layout(C, reached, reached, false)) return R(kRuntimeError);
  }
  // the call stack's growth is given back (hostcall.cpp shrink_stack)
  if (!shrink_stack(C)) return R(kRuntimeError);
  // the whole reserved layout: pages a lane grows into within it must read zero
  const uint32_t init_words = C->mem_words;
  (void)hipEventRecord(C->ev0, C->stream);
  if (!pool_reset(C)) return R(kRuntimeError);
  // after a run the memory kernel's write-mark path resets the instance state as well
  const bool fused = P.has_mem && !C->mem_fresh && init_words;
  // ... or, when that kernel is all this Reset launches (4-byte granules, no per-lane
  // tables, no memories past the first, no start function, no timing asked), the next
  // interpreter launch does it wave by wave (batch_kernel.hip fused_reset): one kernel and
  // one launch gap less per Reset + Run. A host accessor before that launch does it first
  // (settle). WB_FUSED_RESET=0 keeps the separate kernel.
  const char *fre = getenv("WB_FUSED_RESET");
  C->reset_deferred = false;
  const bool defer = fused && C->mlog == 0 && !P.mut_tables && P.xmems.empty() && P.start_func < 0 &&
                     !KernelSeconds && !(C->conf.CostLimit && C->init_exceeded) && !(fre && fre[0] == '0');
  if (defer) {
    C->reset_deferred = true;
  } else if (P.has_mem &&
      !C->hip_ok(wb_launch_mem_init(C->mem.ptr, C->image.ptr, C->image_words, init_words,
                                    C->mem_words, C->nwaves, C->lstate.ptr, C->ls_slots,
                                    C->mem_fresh ? 1u : 0u, C->mlog, fused ? 1u : 0u, C->global_init.ptr, P.mem_min,
                                    C->init_dropped, C->init_cost, C->stream), "mem init"))
    return R(kRuntimeError);
  C->mem_fresh = false;   // from now on every lane's write mark (LS_HWM) is valid
  // per-lane tables (instantiate/table.cpp + elem.cpp): every lane starts from the image
  if (P.mut_tables &&
      !C->hip_ok(wb_launch_mem_init(C->ltab.ptr, C->tab_image.ptr, P.tab_words, P.tab_words,
                                    P.tab_words, C->nwaves, nullptr, 0, 1u, 0u, 0u, nullptr, 0, 0, 0,
                                    C->stream), "table init"))
    return R(kRuntimeError);
  // memories past the first: zeros + their active data segments, initial sizes
  if (!P.xmems.empty() &&
      ((C->xwords && !C->hip_ok(wb_launch_mem_init(C->xmem.ptr, C->ximage.ptr, C->xwords, C->xwords,
                                                    C->xwords, C->nwaves, nullptr, 0, 1u, C->xlog, 0u, nullptr,
                                                    0, 0, 0, C->stream), "memory init")) ||
       !C->hip_ok(hipMemcpyAsync(C->xpages.ptr, C->xpages0.data(), C->xpages0.size() * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, C->stream), "memory sizes")))
    return R(kRuntimeError);
  // gas: instantiation's constant expressions are priced first (module.cpp order); one
  // past the limit fails the instantiation like the reference's VM::instantiate
  if (C->conf.CostLimit && C->init_exceeded)
    return R(C->fail(0x03, "instantiation exceeds the cost limit (constant expressions)"));
  if (!fused && !C->hip_ok(wb_launch_state_init(C->lstate.ptr, C->ls_slots, C->nwaves, C->global_init.ptr,
                                                P.mem_min, C->init_dropped, C->init_cost, C->stream),
                           "state init"))
    return R(kRuntimeError);
  (void)hipEventRecord(C->ev1, C->stream);
  // without a start function and without a request for the time, the next launch on the
  // stream orders after this one: no host round trip (errors surface at the next sync)
  double secs = 0;
  C->reset_pending = true;   // host accessors settle() before touching instance state
  if (KernelSeconds || P.start_func >= 0) {
    C->reset_pending = false;
    if (!C->hip_ok(hipStreamSynchronize(C->stream), "mem init")) return R(kRuntimeError);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, C->ev0, C->ev1);
    secs = ms * 1e-3;
  }
  // module.cpp:160-170: the start function runs as the last step of instantiation; a
  // lane whose start function traps keeps that ErrCode as its instance status
  if (P.start_func >= 0) {
    double ks = 0;
    uint8_t e = launch_exec(C, P.funcs[P.start_func].entry_pc, true, &ks);
    if (e) return R(e);
    secs += ks;
    // the start function takes no input, so every lane ends alike: a trap there fails
    // the instantiation itself, reported like the reference's VM::instantiate
    std::vector<uint8_t> st(C->n);
    if (!C->hip_ok(hipMemcpy(st.data(), C->status.ptr, C->n, hipMemcpyDeviceToHost), "status"))
      return R(kRuntimeError);
    for (uint8_t c : st)
      if (c) return R(C->fail(c, "start function trapped (ErrCode 0x" + hexbyte(c) + ")"));
  }
  if (KernelSeconds) *KernelSeconds = secs;
  C->ran = false;
  return R(0);
}

WasmEdge_Result WasmEdge_BatchRun(WasmEdge_BatchContext *C, double *KernelSeconds) {
  if (!C) return R(kWrongVMWorkflow);
  if (!C->shards.empty()) return wbm::run(C, KernelSeconds);
  DevScope dev(C);
  if (C->func < 0) return R(C->fail(kWrongVMWorkflow, "BatchSetArgs not called"));
  const wb::FuncInfo &F = C->prog.funcs[C->func];
  if (F.imported) return R(C->fail(kRuntimeError, "exported function is a host import"));
  const bool measure = C->trial == 1 || C->trial == 3;
  double ks = 0;
  uint8_t e = launch_exec(C, F.entry_pc, false, KernelSeconds || measure ? &ks : nullptr);
  if (e) return R(e);
  if (KernelSeconds) *KernelSeconds = ks;
  if (C->trial == 5) C->trial = 1;   // (the warm-up run of the layout trial)
  else if (measure && (e = layout_trial(C, ks))) return R(e);
  C->ran = true;
  return R(0);
}

WasmEdge_Result WasmEdge_BatchResults(WasmEdge_BatchContext *C, WasmEdge_Value *Returns,
                                      const uint32_t ReturnLen, uint8_t *PerInstance,
                                      uint64_t *InstrCounts) {
  if (!C) return R(kWrongVMWorkflow);
  if (!C->shards.empty()) return wbm::results(C, Returns, ReturnLen, PerInstance, InstrCounts);
  if (!C->ran) return R(C->fail(kWrongVMWorkflow, "BatchRun not called"));
  std::vector<uint8_t> st(C->n);
  if (!C->hip_ok(hipMemcpy(st.data(), C->status.ptr, C->n, hipMemcpyDeviceToHost), "status"))
    return R(kRuntimeError);
  if (PerInstance) memcpy(PerInstance, st.data(), C->n);
  if (InstrCounts &&
      !C->hip_ok(hipMemcpy(InstrCounts, C->counts.ptr, size_t(C->n) * 8, hipMemcpyDeviceToHost), "counts"))
    return R(kRuntimeError);
  if (Returns && ReturnLen) {
    uint32_t rc = C->result_cells;
    std::vector<uint32_t> cells(size_t(C->n) * (rc ? rc : 1));
    if (rc && !C->hip_ok(hipMemcpy(cells.data(), C->results.ptr, cells.size() * 4,
                                   hipMemcpyDeviceToHost), "results"))
      return R(kRuntimeError);
    for (uint32_t i = 0; i < C->n; i++) {
      uint32_t at = 0;
      for (uint32_t k = 0; k < C->result_types.size(); k++) {
        uint8_t ty = C->result_types[k];
        uint128_t v = 0;
        for (uint32_t q = 0; q < cells_of_value(ty); q++)
          v |= uint128_t(cells[size_t(i) * rc + at++]) << (32 * q);
        if (k < ReturnLen) {
          WasmEdge_Value &out = Returns[size_t(i) * ReturnLen + k];
          out.Value = st[i] != 0 ? 0 : ty == wb::EXTERNREF ? C->xref_out(uint32_t(v)) : v;
          out.Type = static_cast<enum WasmEdge_ValType>(ty);
        }
      }
    }
  }
  return R(0);
}

WasmEdge_Result WasmEdge_BatchExecute(WasmEdge_BatchContext *C, const WasmEdge_String FuncName,
                                      const WasmEdge_Value *Params, const uint32_t ParamLen,
                                      WasmEdge_Value *Returns, const uint32_t ReturnLen,
                                      uint8_t *PerInstance, uint64_t *InstrCounts) {
  if (!C) return R(kWrongVMWorkflow);
  WasmEdge_Result r = WasmEdge_BatchSetArgs(C, FuncName, Params, ParamLen);
  if (r.Code) return r;
  r = WasmEdge_BatchRun(C, nullptr);
  if (r.Code) return r;
  return WasmEdge_BatchResults(C, Returns, ReturnLen, PerInstance, InstrCounts);
}

WasmEdge_Result WasmEdge_BatchMemoryHash(WasmEdge_BatchContext *C, uint64_t *Hashes) {
  if (!C) return R(kWrongVMWorkflow);
  if (!C->shards.empty()) return wbm::gather_u64(C, Hashes, WasmEdge_BatchMemoryHash);
  DevScope dev(C);
  if (!C->settle()) return R(kRuntimeError);
  // the grid covers the largest memory of the batch (a block per page and wave)
  uint32_t maxp = 0;
  if (C->prog.has_mem) {
    const size_t row = 64 * sizeof(uint32_t), pitch = size_t(C->ls_slots) * row;
    std::vector<uint32_t> pages(size_t(C->nwaves) * 64);
    if (!C->hip_ok(hipMemcpy2D(pages.data(), row, C->lstate.ptr + LS_PAGES * 64, pitch, row, C->nwaves,
                               hipMemcpyDeviceToHost), "pages"))
      return R(kRuntimeError);
    for (uint32_t i = 0; i < C->n; i++) maxp = std::max(maxp, pages[i]);
  }
  if (!C->hip_ok(wb_launch_mem_hash(C->mem.ptr, C->lstate.ptr, C->ls_slots, C->hashes.ptr,
                                    C->mem_words, C->n, C->mlog, C->pt_w ? C->ptab.ptr : nullptr,
                                    C->pt_w, maxp, C->stream), "hash"))
    return R(kRuntimeError);
  if (!C->hip_ok(hipStreamSynchronize(C->stream), "hash")) return R(kRuntimeError);
  if (!C->hip_ok(hipMemcpy(Hashes, C->hashes.ptr, size_t(C->n) * 8, hipMemcpyDeviceToHost), "hash"))
    return R(kRuntimeError);
  return R(0);
}

uint32_t WasmEdge_BatchGetCompiledRuns(const WasmEdge_BatchContext *C) {
  if (C && !C->shards.empty()) return WasmEdge_BatchGetCompiledRuns(wbm::first(C));
  return C ? C->jit_runs : 0;
}

const char *WasmEdge_BatchGetEngine(const WasmEdge_BatchContext *C) {
  if (!C) return "";
  if (!C->shards.empty()) return WasmEdge_BatchGetEngine(wbm::first(C));
  std::string e;
  if (!C->threaded) e = "compiled-step";
  else if (C->jit_runs) e = std::string("compiled-runs") + (C->simt ? "+simt" : "") + (C->trip ? "+trip" : "");
  else e = C->jit_on ? "threaded-core (compiled runs failed)" : "threaded-core";
  e += C->frame_hbm ? "/hbm-frames" : C->vframe ? "/vgpr-frames" : "/lds-frames";
  if (C->conf.CostLimit) e += "+metered";
  C->engine_desc = e;
  return C->engine_desc.c_str();
}

uint32_t WasmEdge_BatchGetReservedPages(const WasmEdge_BatchContext *C) {
  if (C && !C->shards.empty()) return WasmEdge_BatchGetReservedPages(wbm::first(C));
  return C ? C->rpages : 0;
}

uint32_t WasmEdge_BatchGetExtraMemoryPages(const WasmEdge_BatchContext *C, uint32_t MemIdx) {
  if (C && !C->shards.empty()) return WasmEdge_BatchGetExtraMemoryPages(wbm::first(C), MemIdx);
  if (!C || MemIdx == 0 || size_t(MemIdx) * 2 > C->xinfo_h.size()) return 0;
  return C->xinfo_h[2 * (MemIdx - 1) + 1];
}

uint32_t WasmEdge_BatchGetMemoryGranule(const WasmEdge_BatchContext *C) {
  if (C && !C->shards.empty()) return WasmEdge_BatchGetMemoryGranule(wbm::first(C));
  return C ? 4u << C->mlog : 0;
}

WasmEdge_Result WasmEdge_BatchGetTotalCosts(WasmEdge_BatchContext *C, uint64_t *Costs) {
  if (!C || !Costs) return R(kWrongVMWorkflow);
  if (!C->shards.empty()) return wbm::gather_u64(C, Costs, WasmEdge_BatchGetTotalCosts);
  if (!C->settle()) return R(kRuntimeError);
  const size_t row = 64 * sizeof(uint32_t), pitch = size_t(C->ls_slots) * row;
  std::vector<uint32_t> lo(size_t(C->nwaves) * 64), hi(lo.size());
  if (!C->hip_ok(hipMemcpy2D(lo.data(), row, C->lstate.ptr + LS_COST * 64, pitch, row, C->nwaves,
                             hipMemcpyDeviceToHost), "costs") ||
      !C->hip_ok(hipMemcpy2D(hi.data(), row, C->lstate.ptr + (LS_COST + 1) * 64, pitch, row,
                             C->nwaves, hipMemcpyDeviceToHost), "costs"))
    return R(kRuntimeError);
  for (uint32_t i = 0; i < C->n; i++) Costs[i] = C->conf.CostLimit ? (uint64_t(hi[i]) << 32) | lo[i] : 0;
  return R(0);
}

uint32_t WasmEdge_BatchGetMemoryPages(WasmEdge_BatchContext *C, uint32_t Inst) {
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (C && !C->shards.empty()) return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchGetMemoryPages(s, l) : 0;
  if (!C || Inst >= C->n || !C->prog.has_mem || !C->settle()) return 0;
  uint32_t p = 0;
  const size_t at = (size_t(Inst / 64) * C->ls_slots + LS_PAGES) * 64 + Inst % 64;
  (void)hipMemcpy(&p, C->lstate.ptr + at, 4, hipMemcpyDeviceToHost);
  return p;
}

WasmEdge_Result WasmEdge_BatchGetMemory(WasmEdge_BatchContext *C, uint32_t Inst, uint32_t Off,
                                        uint8_t *Dst, uint32_t Len) {
  if (!C) return R(kWrongVMWorkflow);
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (!C->shards.empty())
    return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchGetMemory(s, l, Off, Dst, Len) : R(kRuntimeError);
  return R(mem_rw(C, Inst, Off, Len, Dst, nullptr));
}

WasmEdge_Result WasmEdge_BatchSetMemory(WasmEdge_BatchContext *C, uint32_t Inst, uint32_t Off,
                                        const uint8_t *Src, uint32_t Len) {
  if (!C) return R(kWrongVMWorkflow);
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (!C->shards.empty())
    return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchSetMemory(s, l, Off, Src, Len) : R(kRuntimeError);
  return R(mem_rw(C, Inst, Off, Len, nullptr, Src));
}

// ---- exported tables and globals (WasmEdge_TableInstance{Get,Set}Data / GetSize,
// WasmEdge_GlobalInstance{Get,Set}Value, lib/api/wasmedge.cpp:2099-2139, 2273-2295),
// per instance; Inst = WASMEDGE_BATCH_ALL_INSTANCES writes every instance
}  // extern "C"
namespace {
int find_named(const std::vector<wb::ExportFunc> &v, const WasmEdge_String &n) {
  const std::string name(n.Buf ? n.Buf : "", n.Length);
  for (const auto &e : v)
    if (e.name == name) return int(e.func);
  return -1;
}
// word `slot` (in [0, stride)) of instance Inst in a [wave][stride][64] buffer
size_t lane_at(uint32_t Inst, size_t stride, size_t slot) {
  return (size_t(Inst / 64) * stride + slot) * 64 + Inst % 64;
}
bool get_lane(WasmEdge_BatchContext *C, const uint32_t *buf, size_t stride, size_t slot,
              uint32_t Inst, uint32_t *v) {
  if (!C->settle()) return false;
  return C->hip_ok(hipMemcpy(v, buf + lane_at(Inst, stride, slot), 4, hipMemcpyDeviceToHost), "read");
}
bool put_lane(WasmEdge_BatchContext *C, uint32_t *buf, size_t stride, size_t slot,
              uint32_t Inst, uint32_t v) {
  if (!C->settle()) return false;
  if (Inst != WASMEDGE_BATCH_ALL_INSTANCES)
    return C->hip_ok(hipMemcpy(buf + lane_at(Inst, stride, slot), &v, 4, hipMemcpyHostToDevice), "write");
  std::vector<uint32_t> row(size_t(C->nwaves) * 64, v);   // one 64-lane row per wave
  return C->hip_ok(hipMemcpy2D(buf + slot * 64, stride * 256, row.data(), 256, 256, C->nwaves,
                               hipMemcpyHostToDevice), "write");
}
}  // namespace
extern "C" {

WasmEdge_Result WasmEdge_BatchTableGetSize(WasmEdge_BatchContext *C, const WasmEdge_String TableName,
                                           uint32_t Inst, uint32_t *Size) {
  if (!C || !Size) return R(kWrongVMWorkflow);
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (!C->shards.empty())
    return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchTableGetSize(s, TableName, l, Size)
                                       : R(C->fail(kRuntimeError, "instance index out of range"));
  const int t = find_named(C->prog.table_exports, TableName);
  if (t < 0) return R(C->fail(kFuncNotFound, "table export not found"));
  if (Inst >= C->n) return R(C->fail(kRuntimeError, "instance index out of range"));
  return R(get_lane(C, C->lstate.ptr, C->ls_slots, LS_GLOBALS + C->prog.global_cells + t, Inst, Size)
               ? 0 : kRuntimeError);
}

WasmEdge_Result WasmEdge_BatchTableGetData(WasmEdge_BatchContext *C, const WasmEdge_String TableName,
                                           uint32_t Inst, WasmEdge_Value *Data, uint32_t Offset) {
  if (!C || !Data) return R(kWrongVMWorkflow);
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (!C->shards.empty())
    return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchTableGetData(s, TableName, l, Data, Offset)
                                       : R(C->fail(kRuntimeError, "instance index out of range"));
  uint32_t size = 0;
  WasmEdge_Result r = WasmEdge_BatchTableGetSize(C, TableName, Inst, &size);
  if (r.Code) return r;
  const wb::Program &P = C->prog;
  const int t = find_named(P.table_exports, TableName);
  if (Offset >= size) return R(kTableOutOfBounds);   // table.h:131-138 getRefAddr
  uint32_t v = 0;
  if (!get_lane(C, C->ltab.ptr, P.tab_words, P.tabinfo[2 * t] + Offset, Inst, &v))
    return R(kRuntimeError);
  Data->Value = P.tables[t].type == wb::EXTERNREF ? C->xref_out(v) : uint128_t(v);
  Data->Type = static_cast<enum WasmEdge_ValType>(P.tables[t].type);
  return R(0);
}

WasmEdge_Result WasmEdge_BatchTableSetData(WasmEdge_BatchContext *C, const WasmEdge_String TableName,
                                           uint32_t Inst, WasmEdge_Value Data, uint32_t Offset) {
  if (!C) return R(kWrongVMWorkflow);
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (!C->shards.empty()) {
    if (Inst == WASMEDGE_BATCH_ALL_INSTANCES)   // (every shard's bounds first: all or none)
      return wbm::all(C, [&](WasmEdge_BatchContext *x) { return WasmEdge_BatchTableSetData(x, TableName, Inst, Data, Offset); });
    return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchTableSetData(s, TableName, l, Data, Offset)
                                       : R(C->fail(kRuntimeError, "instance index out of range"));
  }
  const wb::Program &P = C->prog;
  const int t = find_named(P.table_exports, TableName);
  if (t < 0) return R(C->fail(kFuncNotFound, "table export not found"));
  if (uint32_t(Data.Type) != P.tables[t].type) return R(kRefTypeMismatch);
  bool full = false;
  const uint32_t v = P.tables[t].type == wb::EXTERNREF ? C->xref_in(Data.Value, &full) : uint32_t(Data.Value);
  if (full) return R(C->fail(kRuntimeError, "externref intern table full (2^31 - 1 values)"));
  if (P.tables[t].type == wb::FUNCREF && v != 0xFFFFFFFFu && v >= P.funcs.size())
    return R(C->fail(kRuntimeError, "funcref is not a function index of the module"));
  if (Inst == WASMEDGE_BATCH_ALL_INSTANCES) {
    // every lane: bounds against each lane's own size (all lanes checked first)
    std::vector<uint32_t> sizes(size_t(C->nwaves) * 64);
    if (!C->settle()) return R(kRuntimeError);
    const size_t slot = LS_GLOBALS + P.global_cells + t;
    if (!C->hip_ok(hipMemcpy2D(sizes.data(), 256, C->lstate.ptr + slot * 64, size_t(C->ls_slots) * 256,
                               256, C->nwaves, hipMemcpyDeviceToHost), "read"))
      return R(kRuntimeError);
    for (uint32_t i = 0; i < C->n; i++)
      if (Offset >= sizes[i]) return R(kTableOutOfBounds);
  } else {
    uint32_t size = 0;
    WasmEdge_Result r = WasmEdge_BatchTableGetSize(C, TableName, Inst, &size);
    if (r.Code) return r;
    if (Offset >= size) return R(kTableOutOfBounds);   // table.h:141-149 setRefAddr
  }
  return R(put_lane(C, C->ltab.ptr, P.tab_words, P.tabinfo[2 * t] + Offset, Inst, v) ? 0 : kRuntimeError);
}

WasmEdge_Result WasmEdge_BatchGlobalGetValue(WasmEdge_BatchContext *C, const WasmEdge_String GlobalName,
                                             uint32_t Inst, WasmEdge_Value *Value) {
  if (!C || !Value) return R(kWrongVMWorkflow);
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (!C->shards.empty())
    return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchGlobalGetValue(s, GlobalName, l, Value)
                                       : R(C->fail(kRuntimeError, "instance index out of range"));
  const wb::Program &P = C->prog;
  const int g = find_named(P.global_exports, GlobalName);
  if (g < 0) return R(C->fail(kFuncNotFound, "global export not found"));
  if (Inst >= C->n) return R(C->fail(kRuntimeError, "instance index out of range"));
  const uint8_t t = P.global_types[g];
  uint128_t v = 0;
  for (uint32_t q = 0; q < wb::cells_of(t); q++) {
    uint32_t w = 0;
    if (!get_lane(C, C->lstate.ptr, C->ls_slots, LS_GLOBALS + P.global_cell[g] + q, Inst, &w))
      return R(kRuntimeError);
    v |= uint128_t(w) << (32 * q);
  }
  if ((t == wb::FUNCREF || t == wb::EXTERNREF) && uint32_t(v) == 0xFFFFFFFFu) v = 0xFFFFFFFFu;
  if (t == wb::EXTERNREF) v = C->xref_out(uint32_t(v));
  Value->Value = v;
  Value->Type = static_cast<enum WasmEdge_ValType>(t);
  return R(0);
}

WasmEdge_Result WasmEdge_BatchGlobalSetValue(WasmEdge_BatchContext *C, const WasmEdge_String GlobalName,
                                             uint32_t Inst, WasmEdge_Value Value) {
  if (!C) return R(kWrongVMWorkflow);
  WasmEdge_BatchContext *s;
  uint32_t l;
  if (!C->shards.empty()) {
    if (Inst == WASMEDGE_BATCH_ALL_INSTANCES)
      return wbm::all(C, [&](WasmEdge_BatchContext *x) { return WasmEdge_BatchGlobalSetValue(x, GlobalName, Inst, Value); });
    return wbm::route(C, Inst, &s, &l) ? WasmEdge_BatchGlobalSetValue(s, GlobalName, l, Value)
                                       : R(C->fail(kRuntimeError, "instance index out of range"));
  }
  const wb::Program &P = C->prog;
  const int g = find_named(P.global_exports, GlobalName);
  if (g < 0) return R(C->fail(kFuncNotFound, "global export not found"));
  if (Inst >= C->n && Inst != WASMEDGE_BATCH_ALL_INSTANCES)
    return R(C->fail(kRuntimeError, "instance index out of range"));
  // wasmedge.cpp:2286-2295: a constant global or a value of another type is ignored
  const uint8_t t = P.global_types[g];
  if (!P.global_mut[g] || uint32_t(Value.Type) != t) return R(0);
  bool full = false;
  const uint128_t x = t == wb::EXTERNREF ? uint128_t(C->xref_in(Value.Value, &full)) : Value.Value;
  if (full) return R(C->fail(kRuntimeError, "externref intern table full (2^31 - 1 values)"));
  for (uint32_t q = 0; q < wb::cells_of(t); q++)
    if (!put_lane(C, C->lstate.ptr, C->ls_slots, LS_GLOBALS + P.global_cell[g] + q, Inst,
                  uint32_t(x >> (32 * q))))
      return R(kRuntimeError);
  return R(0);
}

WasmEdge_Result WasmEdge_BatchAddHostFunction(WasmEdge_BatchContext *C,
                                              const WasmEdge_String ModuleName,
                                              const WasmEdge_String FuncName,
                                              WasmEdge_BatchHostFunc_t Func, void *Data) {
  return WasmEdge_BatchAddHostFunctionWithCost(C, ModuleName, FuncName, Func, Data, 0);
}

WasmEdge_Result WasmEdge_BatchAddHostFunctionWithCost(WasmEdge_BatchContext *C,
                                                      const WasmEdge_String ModuleName,
                                                      const WasmEdge_String FuncName,
                                                      WasmEdge_BatchHostFunc_t Func, void *Data,
                                                      uint64_t Cost) {
  if (!C || !Func) return R(kWrongVMWorkflow);
  if (!C->shards.empty())
    return wbm::all(C, [&](WasmEdge_BatchContext *x) {
      return WasmEdge_BatchAddHostFunctionWithCost(x, ModuleName, FuncName, Func, Data, Cost);
    });
  const std::string mod(ModuleName.Buf ? ModuleName.Buf : "", ModuleName.Length);
  const std::string name(FuncName.Buf ? FuncName.Buf : "", FuncName.Length);
  // every import of that (module, name) binds to it, as an import object would
  for (uint32_t f = 0; f < C->prog.n_imported; f++)
    if (C->prog.funcs[f].import_module == mod && C->prog.funcs[f].import_name == name)
      C->hosts[f] = WasmEdge_BatchContext::HostFn{Func, Data, Cost};
  return R(0);
}

uint32_t WasmEdge_BatchMemoryGetInstance(const WasmEdge_BatchMemoryContext *M) {
  return M ? M->ctx->gid(M->inst) : 0;   // (the batch-wide id, on a multi-device batch too)
}

WasmEdge_Result WasmEdge_BatchMemoryGetData(const WasmEdge_BatchMemoryContext *M, uint8_t *Data,
                                            const uint32_t Offset, const uint32_t Length) {
  if (!M) return R(kWrongVMWorkflow);
  if (M->view) return R(M->view->rw(M->inst % 64, Offset, Length, Data, nullptr));
  return R(mem_rw(M->ctx, M->inst, Offset, Length, Data, nullptr));
}

WasmEdge_Result WasmEdge_BatchMemorySetData(WasmEdge_BatchMemoryContext *M, const uint8_t *Data,
                                            const uint32_t Offset, const uint32_t Length) {
  if (!M) return R(kWrongVMWorkflow);
  if (M->view) return R(M->view->rw(M->inst % 64, Offset, Length, nullptr, Data));
  return R(mem_rw(M->ctx, M->inst, Offset, Length, nullptr, Data));
}

uint32_t WasmEdge_BatchGetInstanceCount(const WasmEdge_BatchContext *C) { return C ? C->n : 0; }

// the marker keeps the hash findable in the file without loading it (srchash.py)
static const char kBuildHash[] = "WB_SRC_HASH=" WB_SRC_HASH;
const char *WasmEdge_BatchGetBuildHash(void) { return kBuildHash + 12; }


uint32_t WasmEdge_BatchGetCodeSize(const WasmEdge_BatchContext *C) {
  if (C && !C->shards.empty()) return WasmEdge_BatchGetCodeSize(wbm::first(C));
  return C ? uint32_t(C->prog.code.size()) : 0;
}

const char *WasmEdge_BatchGetLastError(const WasmEdge_BatchContext *C) {
  return C ? C->last_error.c_str() : g_last_create_error.c_str();
}

#ifdef WB_STATS
// profiling builds only: per-wave counters of the last launch, [waves][16] (batch_kernel.hip)
__attribute__((visibility("default"))) uint32_t wb_stats_read(WasmEdge_BatchContext *C,
                                                              uint64_t *out) {
  if (!C || !C->stats) return 0;
  (void)hipMemcpy(out, C->stats, (size_t(C->nwaves) * 32 + 1024) * sizeof(uint64_t), hipMemcpyDeviceToHost);
  return C->nwaves;
}
#endif

void WasmEdge_BatchInterrupt(WasmEdge_BatchContext *C) {
  if (C && !C->shards.empty()) {
    for (WasmEdge_BatchContext *s : C->shards)
      if (s) WasmEdge_BatchInterrupt(s);
    return;
  }
  if (!C || !C->stop) return;
  static const uint32_t one = 1;
  (void)hipMemcpyAsync(C->stop, &one, 4, hipMemcpyHostToDevice, C->ctl_stream);
  (void)hipStreamSynchronize(C->ctl_stream);
  C->stop_dirty.store(true);   // (after the write landed: the next run clears it)
}

void WasmEdge_BatchDelete(WasmEdge_BatchContext *C) {
  if (!C) return;
  if (!C->shards.empty()) {
    wbm::destroy(C);
    return;
  }
  DevScope dev(C);
  if (C->stream) (void)hipStreamSynchronize(C->stream);
  if (C->ctl_stream) (void)hipStreamDestroy(C->ctl_stream);
  if (C->order_stream) {
    (void)hipStreamSynchronize(C->order_stream);
    (void)hipStreamDestroy(C->order_stream);
  }
  if (C->ev_order) (void)hipEventDestroy(C->ev_order);
  if (C->stop) (void)hipFree(C->stop);
  if (C->parked_h) (void)hipHostFree(C->parked_h);
  if (C->stats) (void)hipFree(C->stats);
  if (C->ev0) (void)hipEventDestroy(C->ev0);
  if (C->ev1) (void)hipEventDestroy(C->ev1);
  hipStream_t s = C->stream;
  for (const auto &ch : C->pool_chunks) (void)hipFree(ch.first);
  delete C;
  if (s) (void)hipStreamDestroy(s);
}

}  // extern "C"
