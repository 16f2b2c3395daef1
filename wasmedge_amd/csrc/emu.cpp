// emu.cpp -- TEST-ONLY host emulator of the DBC interpreter. It compiles the very same
// dbc_step.inc the gfx950 kernel runs (one lane at a time, contiguous per-lane memory)
// so tests can check the lowering and the per-op code against the oracle on a CPU.
// It is built into a separate library (libwasmedge_batch_emu.so) that the product never
// loads; the product path (libwasmedge_batch.so) has no CPU execution path.
#define WB_MSHIFT 0
#define WB_MARK(ea, n) ((void)0)   // the emulator re-creates memory per instance
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "dbc_ops.h"
#include "frontend.h"
#include "kparams.h"
#include "wasi_impl.h"

static std::string g_err;
static uint64_t *g_hist = nullptr;   // optional per-op dispatch histogram (tuning aid)
static uint64_t *g_pchist = nullptr; // optional per-pc dispatch histogram (tuning aid)
static uint32_t g_pchist_n = 0;
static uint32_t *g_trace = nullptr;  // optional per-lane dispatch pc trace (scheduler studies)
static uint64_t g_trace_cap = 0, g_trace_len = 0, *g_trace_lens = nullptr;
// Host-import callback of the emulator (the batched library's yield path, run inline):
// returns 0 and writes the result cells, or an ErrCode that ends the instance.
typedef int (*wb_emu_host_t)(uint32_t inst, uint32_t func, const uint32_t *args,
                             uint32_t *rets, uint8_t *mem, uint64_t mem_bytes);
static wb_emu_host_t g_host = nullptr;
static uint64_t g_cost_limit = ~0ull;   // gas limit (0 = none)
static bool g_tail_call = false;      // TailCall proposal (wb_emu_set_tail_call)
static bool g_multi_memory = false;   // MultiMemories proposal (wb_emu_set_multi_memory)
static std::vector<uint64_t> g_cost_tab;   // cost per OpCode (empty: the unit table)
static std::vector<uint64_t> g_costs;      // per instance: its gas total after the last run
static std::vector<wb::HostImport> g_imports;   // provided tables / memories / globals
// the library's WASI subset (wasi_impl.h), bound before g_host when on
static bool g_wasi = false;
static wbw::Env g_wasi_env;
static std::vector<wbw::Lane> g_wasi_lanes;
struct EmuMem final : wbw::MemIO {
  uint8_t *mb; uint64_t bytes; bool has;
  bool present() override { return has; }
  uint64_t size() override { return bytes; }
  bool read(uint32_t off, uint32_t len, uint8_t *dst) override {
    if (uint64_t(off) + len > bytes) return false;
    memcpy(dst, mb + off, len);
    return true;
  }
  bool write(uint32_t off, uint32_t len, const uint8_t *src) override {
    if (uint64_t(off) + len > bytes) return false;
    memcpy(mb + off, src, len);
    return true;
  }
};

extern "C" {

__attribute__((visibility("default"))) const char *wb_emu_last_error() { return g_err.c_str(); }

// Count dispatches per DBC op into h[DBC_NUM_OPS] during later wb_emu_execute calls (NULL: off).
__attribute__((visibility("default"))) void wb_emu_set_histogram(uint64_t *h) { g_hist = h; }
__attribute__((visibility("default"))) void wb_emu_set_pc_histogram(uint64_t *h, uint32_t n) { g_pchist = h; g_pchist_n = n; }
// Record every dispatched pc into buf[cap], lane after lane; lens[inst] = its entry count
// (NULL: off). Lanes run independently, so a lane's pc sequence does not depend on how a
// wave schedules its lanes: tools/sched_sim.c replays these traces under scheduler policies.
__attribute__((visibility("default"))) void wb_emu_set_pc_trace(uint32_t *buf, uint64_t cap, uint64_t *lens) {
  g_trace = buf; g_trace_cap = cap; g_trace_len = 0; g_trace_lens = lens;
}
__attribute__((visibility("default"))) uint32_t wb_emu_num_ops() { return OP_DBC_NUM_OPS; }
__attribute__((visibility("default"))) void wb_emu_set_host(wb_emu_host_t h) { g_host = h; }
// the TailCall proposal for modules loaded from now on (WasmEdge_BatchConfigure::TailCall)
__attribute__((visibility("default"))) void wb_emu_set_tail_call(int on) { g_tail_call = on != 0; }
// ... and the MultiMemories proposal (WasmEdge_BatchConfigure::MultiMemories)
__attribute__((visibility("default"))) void wb_emu_set_multi_memory(int on) { g_multi_memory = on != 0; }
__attribute__((visibility("default"))) void wb_emu_set_cost_limit(uint64_t l) { g_cost_limit = l ? l : ~0ull; }
// WasmEdge_StatisticsSetCostTable (statistics.h:59-66): `len` entries, the rest 0;
// tab = NULL and len = 0: back to the default unit table
__attribute__((visibility("default"))) void wb_emu_set_cost_table(const uint64_t *tab, uint32_t len) {
  g_cost_tab.clear();
  if (!tab && !len) return;
  g_cost_tab.assign(65536, 0ull);
  for (uint32_t k = 0; k < len && k < 65536; k++) g_cost_tab[k] = tab[k];
}
__attribute__((visibility("default"))) void wb_emu_clear_imports() { g_imports.clear(); }
__attribute__((visibility("default"))) void wb_emu_add_import(const char *mod, const char *name, uint32_t kind,
                                                              uint32_t type, uint32_t mut, uint32_t min,
                                                              uint32_t max, uint32_t has_max,
                                                              const uint32_t *value) {
  wb::HostImport h;
  h.module = mod; h.name = name; h.kind = uint8_t(kind); h.type = uint8_t(type); h.mut = mut != 0;
  h.min = min; h.max = max; h.has_max = has_max != 0;
  for (int q = 0; q < 4; q++) h.value[q] = value ? value[q] : 0u;
  g_imports.push_back(h);
}
__attribute__((visibility("default"))) void wb_emu_get_costs(uint64_t *out, uint32_t n) {
  for (uint32_t k = 0; k < n && k < g_costs.size(); k++) out[k] = g_costs[k];
}
// WASI subset on (args/envs shared by every instance) or off; outputs per instance of the
// last wb_emu_execute
__attribute__((visibility("default"))) void wb_emu_set_wasi(int on, const char *const *args, uint32_t nargs,
                                                            const char *const *envs, uint32_t nenvs) {
  g_wasi = on != 0;
  g_wasi_env.args.assign(args, args + nargs);
  g_wasi_env.envs.assign(envs, envs + nenvs);
}
// preopen guest names (fds 3, 4, ...) and per-instance command lines for the next
// wb_emu_execute (an instance without its own args uses the shared ones)
static std::vector<std::vector<std::string>> g_wasi_inst_args;
static std::vector<bool> g_wasi_inst_own;
__attribute__((visibility("default"))) void wb_emu_set_wasi_preopens(const char *const *dirs, uint32_t n) {
  g_wasi_env.preopens.clear();
  g_wasi_env.host.clear();
  for (uint32_t k = 0; k < n; k++) wbw::add_preopen(g_wasi_env, dirs[k]);
}
// reproducible fd numbers / random_get / clocks (WasmEdge_BatchWASISetDeterministic)
__attribute__((visibility("default"))) void wb_emu_set_wasi_deterministic(int on, uint64_t seed, uint64_t clock_ns) {
  g_wasi_env.seed = seed;
  g_wasi_env.fixed_clock = on != 0;
  g_wasi_env.clock_ns = clock_ns;
}
__attribute__((visibility("default"))) void wb_emu_set_instance_args(uint32_t inst, const char *const *args, uint32_t n) {
  if (inst >= g_wasi_inst_args.size()) { g_wasi_inst_args.resize(inst + 1); g_wasi_inst_own.resize(inst + 1, false); }
  g_wasi_inst_args[inst].assign(args, args + n);
  g_wasi_inst_own[inst] = true;
}
__attribute__((visibility("default"))) void wb_emu_clear_instance_args() {
  g_wasi_inst_args.clear();
  g_wasi_inst_own.clear();
}
__attribute__((visibility("default"))) uint32_t wb_emu_wasi_output(uint32_t inst, uint32_t fd, uint8_t *buf, uint32_t len) {
  if (inst >= g_wasi_lanes.size() || (fd != 1 && fd != 2)) return 0;
  const std::string &o = g_wasi_lanes[inst].out[fd - 1];
  if (buf) memcpy(buf, o.data(), std::min<size_t>(len, o.size()));
  return uint32_t(o.size());
}
__attribute__((visibility("default"))) uint32_t wb_emu_wasi_exit_code(uint32_t inst) {
  return inst < g_wasi_lanes.size() ? g_wasi_lanes[inst].exit_code : 0;
}

// Returns ErrCode of the call; per-instance outputs like WasmEdge_BatchExecute.
// params: [n][param cells] u32; results: [n][result cells] u32.
__attribute__((visibility("default"))) int wb_emu_execute(
    const uint8_t *wasm, uint32_t len, const char *func, uint32_t n, const uint32_t *params,
    uint32_t *results, uint8_t *statuses, uint64_t *counts, uint64_t *hashes,
    uint32_t max_pages, uint32_t gs_depth, uint64_t max_steps) {
  wb::Program P;
  uint8_t ec = 0;
  g_err = wb::load_program(wasm, len, P, &ec, g_cost_limit != ~0ull, &g_imports, g_tail_call,
                           g_multi_memory);
  if (!g_err.empty()) return ec ? ec : 2;
  int f = wb::find_export(P, func);
  if (f < 0) { g_err = "function not found"; return 0x05; }
  const wb::FuncInfo &F = P.funcs[f];
  const wb::FuncType &T = P.types[F.type];
  uint32_t pcells = 0, rcells = 0;
  for (uint8_t t : T.params) pcells += wb::cells_of(t);
  for (uint8_t t : T.results) rcells += wb::cells_of(t);
  // page limit as the library's (memory.h:88-115): 65536, the module's max, max_pages
  uint32_t limit = 65536;
  if (P.mem_has_max) limit = std::min(limit, P.mem_max);
  if (max_pages) limit = std::min(limit, max_pages);
  if (limit < P.mem_min) limit = P.mem_min;
  if (!P.has_mem) limit = 0;
  if (!gs_depth) gs_depth = 4096;
  std::vector<DFunc> fv;
  for (const auto &fi : P.funcs) fv.push_back(DFunc{fi.imported ? 0xFFFFFFFFu : fi.entry_pc, P.type_canon[fi.type]});
  std::vector<uint8_t> pool;
  std::vector<uint32_t> doff, dlen;
  std::vector<uint32_t> init_dropped((P.datas.size() + 31) / 32 + 1, 0u);   // a bit per data segment
  for (size_t k = 0; k < P.datas.size(); k++) {
    doff.push_back(uint32_t(pool.size()));
    dlen.push_back(uint32_t(P.datas[k].bytes.size()));
    pool.insert(pool.end(), P.datas[k].bytes.begin(), P.datas[k].bytes.end());
    if (P.datas[k].active) init_dropped[k >> 5] |= 1u << (k & 31);
  }
  KParams p{};
  p.code = P.code.data(); p.brtab = P.brtab.data(); p.vconst = P.vconst.data();
  p.funcs = fv.data(); p.table = P.table0.data(); p.global_init = P.global_init.data();
  p.data_pool = pool.data(); p.data_off = doff.data(); p.data_len = dlen.data();
  p.results = results; p.param_cells = pcells; p.result_cells = rcells;
  p.global_cells = P.global_cells; p.total_cells = P.total_cells();
  p.table_size = uint32_t(P.table0.size()); p.mem_max_pages = limit;
  p.gs_depth = gs_depth;
  p.mut_tables = P.mut_tables ? 1u : 0u; p.ntables = P.ntables; p.tab_words = P.tab_words;
  p.tabinfo = P.tabinfo.data(); p.elem_pool = P.elem_pool.data();
  p.elem_off = P.elem_off.data(); p.elem_len = P.elem_len.data();
  std::vector<uint32_t> ltabv, tsz;   // this instance's tables (per-lane table mode)
  std::vector<uint32_t> edrop;
#define TSIZE(t) tsz[(uint32_t)(t)]
#define TENT(t, i) ltabv[P.tabinfo[2u * (t)] + (i)]
#define ELEM_DROPPED(e) ((edrop[(e) >> 5] >> ((e) & 31u)) & 1u)
#define SET_ELEM_DROPPED(e) (edrop[(e) >> 5] |= 1u << ((e) & 31u))
#define DATA_DROPPED(s) ((dropped[(s) >> 5] >> ((s) & 31u)) & 1u)
#define SET_DATA_DROPPED(s) (dropped[(s) >> 5] |= 1u << ((s) & 31u))
  // a table.grow past table t's capacity: the tables widen as the library's host service
  // does (hostcall.cpp widen_tables: at least double, within table_widen_limit), this
  // instance's entries and the image later instances start from relaid out together
  const char *twe = getenv("WB_TABLE_WIDEN");   // (=0: the first capacity stays, as the library's)
  const bool no_widen = twe && twe[0] == '0';
  auto twiden = [&](uint32_t t, uint64_t want) {
    if (no_widen || want > wb::table_widen_limit(P.tables[t])) return;
    const uint64_t cap = std::min<uint64_t>(wb::table_widen_limit(P.tables[t]),
                                            std::max<uint64_t>(want, 2ull * P.tabinfo[2 * t + 1]));
    std::vector<uint32_t> info(P.tabinfo.size());
    uint64_t words = 0;
    for (uint32_t u = 0; u < P.ntables; u++) {
      info[2 * u] = uint32_t(words);
      info[2 * u + 1] = u == t ? uint32_t(cap) : P.tabinfo[2 * u + 1];
      words += info[2 * u + 1];
    }
    std::vector<uint32_t> nl(words, 0xFFFFFFFFu), ni(words, 0xFFFFFFFFu);
    for (uint32_t u = 0; u < P.ntables; u++) {
      const uint32_t f = P.tabinfo[2 * u], c = P.tabinfo[2 * u + 1];
      std::copy(ltabv.begin() + f, ltabv.begin() + f + c, nl.begin() + info[2 * u]);
      std::copy(P.tab_image.begin() + f, P.tab_image.begin() + f + c, ni.begin() + info[2 * u]);
    }
    ltabv.swap(nl);
    P.tab_image.swap(ni);
    P.tabinfo.swap(info);
    P.tab_words = uint32_t(words);
    p.tabinfo = P.tabinfo.data();
    p.tab_words = P.tab_words;
  };
#define WB_TWIDEN(t, want) twiden((t), (want))
  std::vector<uint32_t> frame(P.total_cells() + 8), gstack(gs_depth);
  std::vector<uint32_t> memv;
  // gas metering: per DBC prefix sums of its instructions' costs (unit table by default)
  const bool metered = g_cost_limit != ~0ull;
  std::vector<uint64_t> unit, cpool;
  std::vector<uint32_t> coff;
  if (g_cost_tab.empty()) unit.assign(65536, 1ull);
  const uint64_t *tab = g_cost_tab.empty() ? unit.data() : g_cost_tab.data();
  bool init_exceeded = false;
  const uint64_t init_cost = metered ? wb::build_cost_pool(P, tab, g_cost_limit, coff, cpool, &init_exceeded) : 0;
  const uint64_t c_else = tab[0x05];
  uint64_t cost = 0;
  g_costs.assign(n, 0);
  // imports served by the WASI subset (wasi_impl.h), per function index
  std::vector<int> wasi_fn(P.funcs.size(), -1);
  g_wasi_lanes.assign(g_wasi ? n : 0, wbw::Lane{});
  for (uint32_t k = 0; k < g_wasi_lanes.size(); k++) g_wasi_lanes[k].index = k;
  for (uint32_t k = 0; g_wasi && k < n && k < g_wasi_inst_own.size(); k++)
    if (g_wasi_inst_own[k]) { g_wasi_lanes[k].own_args = true; g_wasi_lanes[k].args = g_wasi_inst_args[k]; }
  for (uint32_t f = 0; g_wasi && f < P.n_imported; f++)
    if (P.funcs[f].import_module == "wasi_snapshot_preview1")
      wasi_fn[f] = wbw::lookup(P.funcs[f].import_name, P.types[P.funcs[f].type].params,
                               P.types[P.funcs[f].type].results);
  for (uint32_t inst = 0; inst < n; inst++) {
    // instantiate: memory image + globals
    memv.assign(size_t(P.mem_min) << 14, 0u);   // (memory.grow resizes it)
    uint8_t *mb = reinterpret_cast<uint8_t *>(memv.data());
    for (const auto &d : P.datas)
      if (d.active && !d.mem && !d.bytes.empty()) memcpy(mb + d.offset, d.bytes.data(), d.bytes.size());
    // memories past the first (MultiMemories): their own vectors, limits as memory 0's
    std::vector<std::vector<uint32_t>> xmemv(P.xmems.size());
    std::vector<uint32_t> xpg(P.xmems.size()), xlim(P.xmems.size());
    for (size_t k = 0; k < P.xmems.size(); k++) {
      xpg[k] = P.xmems[k].min;
      xlim[k] = std::min<uint32_t>(65536, P.xmems[k].has_max ? P.xmems[k].max : 65536);
      if (max_pages) xlim[k] = std::min(xlim[k], max_pages);
      xmemv[k].assign(size_t(xpg[k]) << 14, 0u);
    }
    for (const auto &d : P.datas)
      if (d.active && d.mem && !d.bytes.empty())
        memcpy(reinterpret_cast<uint8_t *>(xmemv[d.mem - 1].data()) + d.offset, d.bytes.data(), d.bytes.size());
#define XMEM(k) xmemv[(k) - 1u].data()
#define XPAGES(k) xpg[(k) - 1u]
#define XLIMIT(k) xlim[(k) - 1u]
#define XGROW(k, cur, n) do { xmemv[(k) - 1u].resize(size_t((cur) + (n)) << 14, 0u); xpg[(k) - 1u] = (cur) + (n); } while (0)
    uint32_t *fr = frame.data(), *gs = gstack.data(), *mem = memv.data();
#define CELL(x) fr[(uint32_t)(x)]
#define R32(x) CELL(x)
#define W32(x, v) (CELL(x) = (uint32_t)(v))
#define R64(x) ((uint64_t)CELL(x) | ((uint64_t)CELL((x) + 1) << 32))
#define W64(x, v) do { const uint64_t _v = (v); CELL(x) = (uint32_t)_v; CELL((x) + 1) = (uint32_t)(_v >> 32); } while (0)
#define GS(slot) gs[(size_t)(slot)]
#define GS_RD(s) GS(s)
#define GS_WR(s, v) (GS(s) = (v))
#define GS_FAST(hi) true
#define WB_UNIFORM(x) (x)   // (one lane)
#define GSF_BASE(s) (&GS(s))
#define GS_PTR uint32_t *const
#define GS_CPTR const uint32_t *const
#define TRAP(code) do { status = (code); add = (int32_t)cnt8 - (int32_t)post8; } while (0)
#define FINISH() (status = WB_STATUS_OK)
#define JUMP(t, tc) do { npc = (t); add += (tc); jtc = (tc); goto e_next; } while (0)
#define JUMP_LANE(t, tc) JUMP(t, tc)
#define BRANCH(c, t, tc) do { if (c) { npc = (t); add += (tc); jtc = (tc); } goto e_next; } while (0)
#define EXIT_IF_TRAPPED(t) ((void)0)
#define TRAP_CHECK() ((void)0)
#define SLOW_OP() ((void)0)
#define SLOW_IF(c) ((void)0)
#define HOST_YIELD(f, base) do { status = WB_ERR_HOST_CALL; ycall = (f); ybase = (base); } while (0)
#define WB_FAST 0
#define MEM_BYTES ((uint64_t)pages << 16)
#define MEM_PAGES pages
#define WB_GROW(cur, n, res) do { try { memv.resize(size_t((cur) + (n)) << 14, 0u); } catch (...) { break; } \
    mem = memv.data(); mb = reinterpret_cast<uint8_t *>(mem); pages = (cur) + (n); res = (cur); } while (0)
#define W128(c, v) do { for (int _k = 0; _k < 4; _k++) W32((c) + _k, (v)[_k]); } while (0)
#define WLOOP(c, v) W32(c, v)
    uint32_t pages = P.mem_min;
    std::vector<uint32_t> dropped = init_dropped;
    ltabv = P.tab_image;
    tsz.clear();
    for (const auto &t : P.tables) tsz.push_back(t.min);
    edrop = P.init_edropped;
    edrop.resize(edrop.size() + 1, 0u);
    for (uint32_t c = 0; c < P.global_cells; c++) W32(c, P.global_init[c]);
    // one invocation of the function at `entry` on this instance's state
    auto invoke = [&](uint32_t entry, const uint32_t *prm, uint32_t ncells, uint64_t &count) {
      uint32_t status = WB_STATUS_RUNNING, pc = entry, gsp = 0, ycall = 0, ybase = 0;
      for (uint32_t c = 0; c < ncells; c++) W32(P.global_cells + c, prm[c]);
      GS(0) = DBC_EXIT_PC;
      gsp = 1;
      while (status == WB_STATUS_RUNNING) {
        if (max_steps && count >= max_steps) { status = 0x07; break; }
        const uint32_t pcs = pc;
        const DInstr I = P.code[pcs];
        const uint32_t w0 = I.w0, w1 = I.w1, w2 = I.w2, w3 = I.w3;
        const uint32_t op = w0 & 0xFFFFu;
        if (g_hist) g_hist[op]++;
        if (g_pchist && pcs < g_pchist_n) g_pchist[pcs]++;
        if (g_trace && g_trace_len < g_trace_cap) { g_trace[g_trace_len++] = pcs; g_trace_lens[inst]++; }
        const uint32_t cnt8 = (w0 >> 16) & 0xFFu, post8 = (w0 >> 24) & 0x7Fu;
        int32_t add = (int32_t)cnt8, jtc = 0;
        uint32_t npc = pcs + 1;
        const int32_t tcnt = (int32_t)(int16_t)(w2 >> 16);
        // gas as the kernel's slow step (batch_kernel.hip, dbc_ops.h gas_step / gas_tail)
        const uint64_t *cp = metered ? cpool.data() + coff[pcs] : nullptr;
        if (metered && gas_step(cp, 0, cnt8 - post8, g_cost_limit, cost, add)) {
          status = 0x03u;
          goto e_done;
        }
        switch (op) {
#define WB_XMEM_ON 1
#include "dbc_step.inc"
#undef WB_XMEM_ON
        }
      e_next:
        if (metered && (status == WB_STATUS_RUNNING || status == WB_STATUS_OK) &&
            gas_tail(cp, cnt8 - post8, cnt8, jtc, jtc < 0 ? cpool.data() + coff[npc] : nullptr,
                     c_else, g_cost_limit, cost, add))
          status = 0x03u;
      e_done:
        count += (int64_t)add;
        pc = npc;
        const int wfn = status == WB_ERR_HOST_CALL ? wasi_fn[ycall] : -1;
        if (status == WB_ERR_HOST_CALL && (g_host || wfn >= 0)) {   // run the host function inline
          const wb::FuncType &ht = P.types[P.funcs[ycall].type];
          uint32_t rets[64] = {0}, nr = 0;
          for (uint8_t t : ht.results) nr += wb::cells_of(t);
          int e;
          if (wfn >= 0) {
            EmuMem em;
            em.mb = mb; em.bytes = uint64_t(pages) << 16; em.has = P.has_mem;
            uint64_t wa[wbw::kMaxArgs] = {0};
            wbw::args_of_cells(ht.params, &fr[ybase], wa);
            e = wbw::call(wfn, g_wasi_env, g_wasi_lanes[inst], em, wa, &rets[0]);
          } else {
            e = g_host(inst, ycall, &fr[ybase], rets, mb, uint64_t(pages) << 16);
          }
          if (e) { status = uint32_t(e); break; }
          for (uint32_t k = 0; k < nr; k++) W32(ybase + k, rets[k]);
          status = WB_STATUS_RUNNING;
        }
      }
      return status;
    };
    // instantiation ends with the start function (module.cpp:160-170); its count is
    // not part of the invocation's
    uint64_t count = 0, start_count = 0;
    uint32_t status = WB_STATUS_OK;
    // instantiation spends gas too: its constant expressions, then the start function
    cost = init_cost;
    if (init_exceeded) status = 0x03u;
    if (status == WB_STATUS_OK && P.start_func >= 0) {
      p.result_cells = 0;
      status = invoke(P.funcs[P.start_func].entry_pc, nullptr, 0, start_count);
      p.result_cells = rcells;
    }
    if (status == WB_STATUS_OK)
      status = invoke(F.entry_pc, params + size_t(inst) * pcells, pcells, count);
    statuses[inst] = uint8_t(status);
    counts[inst] = count;
    g_costs[inst] = cost;
    if (hashes) {
      uint64_t h = 0, nw = uint64_t(pages) << 13;
      for (uint64_t i = 0; i < nw; i++) {
        uint64_t w = uint64_t(mem[2 * i]) | (uint64_t(mem[2 * i + 1]) << 32);
        h += fmix64(w ^ (i * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull));
      }
      hashes[inst] = h ^ fmix64(uint64_t(pages) + 0x1234567ull);
    }
  }
  return 0;
}

// Disassemble the lowered program (debugging / tests of the lowering).
__attribute__((visibility("default"))) int wb_emu_disasm(const uint8_t *wasm, uint32_t len,
                                                         char *out, uint32_t outlen) {
  wb::Program P;
  uint8_t ec = 0;
  g_err = wb::load_program(wasm, len, P, &ec, false, nullptr, g_tail_call);
  if (!g_err.empty()) return ec ? ec : 2;
  std::string s;
  char buf[160];
  for (size_t k = 0; k < P.code.size(); k++) {
    const DInstr &I = P.code[k];
    snprintf(buf, sizeof buf, "%5zu %-18s cnt=%u post=%u a=%u b=%u c=%u d=%d imm=%u\n", k,
             wb::dop_name(I.w0 & 0xFFFF), (I.w0 >> 16) & 0xFF, I.w0 >> 24, I.w1 & 0xFFFF,
             I.w1 >> 16, I.w2 & 0xFFFF, int(int16_t(I.w2 >> 16)), I.w3);
    s += buf;
  }
  snprintf(buf, sizeof buf, "; globals=%u frame=%u code=%zu divergent_mem=%d\n", P.global_cells,
           P.frame_cells, P.code.size(), int(P.divergent_mem));
  s += buf;
  if (out && outlen) {
    strncpy(out, s.c_str(), outlen - 1);
    out[outlen - 1] = 0;
  }
  return 0;
}

}  // extern "C"
