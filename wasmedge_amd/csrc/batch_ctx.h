// batch_ctx.h -- the batch context shared by the C-ABI translation units
// (batch_api.cpp: create/run/results; hostcall.cpp: the host-import service rounds;
// wasi.cpp: the built-in WASI subset). Host-only; never included by device code.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>
#include <atomic>
#include <memory>
#include <mutex>
#include <unordered_map>

#include "../../include/wasmedge_batch.h"
#include "frontend.h"
#include "tc.h"
#include "kparams.h"
#include "wasi_impl.h"

namespace wbh {

// ErrCodes (include/common/enum.inc)
constexpr uint8_t kRuntimeError = 0x02, kWrongVMWorkflow = 0x04, kFuncNotFound = 0x05,
                  kFuncSigMismatch = 0x83, kTableOutOfBounds = 0x87, kMemoryOutOfBounds = 0x88,
                  kRefTypeMismatch = 0x8E;

inline std::string g_last_create_error;

inline WasmEdge_Result R(uint8_t c) { return WasmEdge_Result{c}; }

inline std::string hexbyte(uint8_t c) {
  const char *d = "0123456789ABCDEF";
  return std::string(1, d[c >> 4]) + d[c & 15];
}

template <typename T>
struct DevBuf {
  T *ptr = nullptr;
  size_t n = 0;
  ~DevBuf() { if (ptr) (void)hipFree(ptr); }
  bool alloc(size_t count) {
    if (ptr) { (void)hipFree(ptr); ptr = nullptr; }
    n = count;
    if (count == 0) return true;
    return hipMalloc(&ptr, sizeof(T) * count) == hipSuccess;
  }
  bool upload(const std::vector<T> &v, hipStream_t s) {
    if (!alloc(v.size() ? v.size() : 1)) return false;
    if (v.empty()) return true;
    return hipMemcpyAsync(ptr, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, s) == hipSuccess;
  }
};

}  // namespace wbh

namespace wbh { struct WaveView; }

// a Reset left to the next launch (batch_kernel.hip fused_reset) done now, as its own
// kernel: for a host accessor or any device work that reads instance state first
bool wbh_reset_now(WasmEdge_BatchContext *C);

struct WasmEdge_BatchMemoryContext {   // one instance's linear memory, for host functions
  WasmEdge_BatchContext *ctx;
  uint32_t inst;
  wbh::WaveView *view;                 // the service round's cached view of its wave (or NULL)
};

struct WasmEdge_BatchContext {
  template <typename T> using DevBuf = wbh::DevBuf<T>;
  wb::Program prog;
  std::vector<wb::HostImport> imports;   // provided tables / memories / globals
  WasmEdge_BatchConfigure conf{};
  uint32_t n = 0, nwaves = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t ctl_stream = nullptr;  // interrupt requests, while `stream` runs a kernel
  uint32_t *stop = nullptr;          // uncached device word polled by the kernel
  uint32_t *parked_h = nullptr, *parked_d = nullptr;   // host-mapped: a lane parked (KParams::parked)
  std::atomic<bool> stop_dirty{false};   // an Interrupt set *stop since the last clear
  uint64_t *stats = nullptr;         // WB_STATS builds: per-wave counters (WB_STATS_OUT)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string last_error;
  mutable std::string engine_desc;   // (WasmEdge_BatchGetEngine's string)
  // module buffers
  DevBuf<DInstr> code;
  DevBuf<TInstr> tcode;           // threaded code for the dispatch core (tc.h)
  bool threaded = true;
  bool vframe = false;            // threaded core with the frame in VGPRs (wb_exec_vf_kernel)
  uint32_t jit_runs = 0;          // compiled straight-line runs (jit.h)
  bool simt = false;              // KParams::simt: the compiled runs schedule diverged lanes
  bool trip = false;              // ... in trip mode (jit.h)
  bool want_simt = false, want_trip = false, jit_on = false;   // (compile_runs inputs)
  std::vector<DInstr> codepad0;   // the module's DBC before compile_runs flags it
  // layout trial (batch_api.cpp layout_trial): 5 = the next run is the warm-up, 1 = the
  // next run measures the module's granule, 2 = the next Reset switches to the other one,
  // 3 = the next run measures that, 4 = the next Reset switches back; 0 = decided
  uint8_t trial = 0;
  uint32_t trial_mlog[2] = {0, 0};   // (the module's granule, the other one)
  int trial_func = -1;
  double trial_rate = 0;
  bool frame_hbm = false;         // frames in HBM (wb_exec_hbm_kernel), KParams::hframe
  DevBuf<uint32_t> hframe;
  // persistent waves (KParams::wave_ctr): the exec kernel's resident blocks for the last
  // launch geometry, and the counter of batch waves taken
  uint32_t cap_threads = 0, cap_blocks = 0;
  size_t cap_lds = 0;
  DevBuf<uint32_t> wave_ctr;
  bool ctr_zero = false;           // wave_ctr is 0 (zeroed by the wave-order kernel)
  hipStream_t order_stream = nullptr;   // the wave-order kernel (overlaps the next Reset)
  hipEvent_t ev_order = nullptr;        // its end; the next persistent launch waits on it
  bool order_pending = false;
  // Longest-first wave order (KParams::wave_order): each persistent launch records every
  // batch wave's run time; the next launch of the same function takes the waves in
  // descending order of it (LPT), so the heavy waves start first instead of wherever their
  // ids put them. Scheduling only: results never depend on it (WB_LPT=0 turns it off).
  DevBuf<uint32_t> wave_ticks, wave_order;
  uint32_t order_pc = 0xFFFFFFFFu;   // entry pc of the launch the order was taken from
  uint64_t order_fp = 0, args_fp = 1;   // its arguments' fingerprint; the staged arguments'
  bool lpt = true;
  uint32_t sched = 1;             // KParams::sched (WB_SCHED=k; 0: min-pc scheduling only)
  DevBuf<uint32_t> loops;         // Program::loops (scheduler)
  DevBuf<uint32_t> brtab, vconst, table, global_init, image, data_off, data_len;
  DevBuf<uint32_t> tab_image, tabinfo, elem_pool, elem_off, elem_len;   // per-lane tables
  DevBuf<DFunc> funcs;
  // gas metering (conf.CostLimit): per-DBC cost prefix sums, the cost of instantiation's
  // constant expressions, the manual `else` cost
  std::vector<uint32_t> cost_off_h;
  std::vector<uint64_t> cost_pool_h;
  DevBuf<uint32_t> cost_off;
  DevBuf<uint64_t> cost_pool;
  uint64_t init_cost = 0, cost_else = 0;
  bool init_exceeded = false;
  DevBuf<uint8_t> data_pool;
  // instance state
  DevBuf<uint32_t> mem, gstack, lstate, params, results, ltab;
  // memories past the first (MultiMemories, KParams::xmem): their device words, every
  // lane's initial image (zeros + active data segments), sizes; at every Reset from
  // ximage / xpages0
  DevBuf<uint32_t> xmem, ximage, xpages, xinfo;
  std::vector<uint32_t> xpages0, xinfo_h;   // xinfo: base word, page limit per memory
  uint32_t xwords = 0;
  // their granule: 4 << xlog bytes (KParams::xlog; batch_api.cpp setup)
  uint32_t xlog = 0;
  // host-import yield path (only allocated when the module imports functions)
  DevBuf<uint32_t> fsave, hcall, hbuf;
  uint32_t hb_cells = 0;
  // a bound import: the function, its Data and its gas cost (HostFunctionBase::Cost)
  struct HostFn { WasmEdge_BatchHostFunc_t fn = nullptr; void *data = nullptr; uint64_t cost = 0; };
  std::vector<HostFn> hosts;      // per function index (imports only)
  uint32_t host_threads = 0;      // service-round worker threads (0 or 1: one, serial)
  // built-in WASI subset (wasi.cpp): args/envs shared by every instance, captured
  // stdout/stderr and the proc_exit code per instance
  struct WasiSlot { WasmEdge_BatchContext *ctx; int fn; };
  wbw::Env wasi_env;
  std::vector<wbw::Lane> wasi_lanes;
  std::vector<WasiSlot> wasi_slots;   // per function index (Data of its HostFn)
  DevBuf<uint8_t> status;
  DevBuf<uint64_t> counts, hashes;
  uint32_t image_words = 0, init_dropped = 0, ls_drop_ext = 0;
  uint32_t mem_max_pages = 0, mem_words = 0, gs_depth = 0, ls_slots = 0, gs_lds = 0;
  // the call stack grows on demand (CallStackCells 0): a call past gs_depth parks, the host
  // doubles the stack (grow_stack) while device memory allows (KParams::gs_grow)
  bool gs_grow = false, gs_grow0 = false;
  uint32_t gs_depth0 = 0;                 // (the depth BatchReset returns the stack to)
  // per-lane tables widen on demand: a table.grow past its capacity parks, the host relays
  // the tables out wider (hostcall.cpp widen_tables; KParams::tg_grow / tlimit)
  bool tg_grow = false;
  DevBuf<uint32_t> tlimit;
  // Paged linear memory (DESIGN.md "Linear memory"): `mem_max_pages` is the page limit
  // (65536, the module's max, MaxMemoryPage); pages [0, rpages) of every lane live in the
  // reserved layout at `mem` (mem_words = rpages * 16384 words per lane), page q >= rpages
  // of wave w in a pool row of 64 lanes x 64 KiB at pt_host[w * pt_w + q - rpages]. Rows
  // come from hipMalloc'ed chunks, zeroed, handed out by the host when a lane parks at a
  // memory.grow past its wave's rows (hostcall.cpp serve_grows) -- the batched
  // Allocator::resize (lib/system/allocator.cpp:101-129), which commits pages on demand.
  uint32_t rpages = 0;
  uint32_t rpages0 = 0;              // rpages at BatchCreate (grow_layout bounds the growth
                                     // past it by MemoryPoolBytes)
  bool grow_host = false;            // the module can grow past rpages
  uint32_t pt_w = 0;                 // page-table width: pool pages per wave it can name
  std::vector<uint64_t> pt_host;     // [nwaves][pt_w] row device addresses (0: none)
  std::vector<uint32_t> pt_n;        // [nwaves] rows each wave holds (pages rpages.. +n)
  DevBuf<uint64_t> ptab;             // the device copy of pt_host
  bool pt_dirty = false;             // pt_host changed since the last upload
  std::vector<uint64_t> pool_free;   // zeroed rows not handed out
  std::vector<std::pair<void *, size_t>> pool_chunks;   // (base, bytes), freed at Delete
  size_t pool_bytes = 0;             // bytes of chunks allocated
  bool pool_used = false;            // rows were handed out since the last Reset
  // device address of word-row `word` (a multiple of 64) of wave `wave`: that word of its
  // 64 lanes, and the rows after it up to the end of its page; nullptr past the wave's rows
  uint32_t *wave_rows(uint32_t wave, uint64_t word) const {
    if (word < mem_words) return mem.ptr + (size_t(wave) * mem_words + word) * 64;
    const uint64_t k = (word >> 14) - rpages;
    if (k >= pt_w) return nullptr;
    const uint64_t a = pt_host[size_t(wave) * pt_w + k];
    return a ? reinterpret_cast<uint32_t *>(a) + size_t(word & 16383u) * 64 : nullptr;
  }
  uint32_t mlog = 0;              // log2(words per memory interleave granule), KParams::mlog
  // current invocation
  int func = -1;
  uint32_t param_cells = 0, result_cells = 0;
  std::vector<uint8_t> result_types;
  bool ran = false;         // a Run completed since the last Reset (results are valid)
  bool mem_fresh = true;    // memory never initialised: the next Reset writes every page
  // A Reset that skipped its host sync left init kernels queued on `stream` (non-blocking,
  // so NOT ordered before the host accessors' synchronous null-stream copies): every host
  // accessor settles first.
  bool reset_pending = false;
  // ... or not even queued: the next launch of the interpreter does it (fused_reset)
  bool reset_deferred = false;

  // Multi-device contexts (WasmEdge_BatchConfigure::Devices, multi.cpp): the parent holds
  // one shard context per entry of Devices (nullptr: no instances there) and routes every
  // call to them; a shard is a whole single-device context over its part of the ids.
  std::vector<WasmEdge_BatchContext *> shards;
  uint32_t part = 0;
  WasmEdge_BatchContext *parent = nullptr;   // (a shard)
  uint32_t shard_g = 0;
  std::mutex *host_mu = nullptr;             // shards: one host service round at a time
  std::mutex own_host_mu;                    // (the parent's, when HostThreads <= 1)
  // the batch-wide instance id of this context's lane `local`
  uint32_t gid(uint32_t local) const;

  // externref values at the boundary (the reference's are host pointers, wasmedge.h:254,318)
  // and the 32-bit refs the device carries: null is 0xFFFFFFFF both sides, a value below
  // 2^31 is its own device ref, a wider one (a pointer) is interned as 0x80000000 + its
  // index here, for the context's life, and given back as the same 64-bit value
  std::vector<uint64_t> xref_vals;
  std::unordered_map<uint64_t, uint32_t> xref_ids;
  std::mutex xref_mu;   // (host functions may run on several threads)
  // *full is set when a wide value finds the intern table full: the call that passed it
  // fails (RuntimeError; a host function's result: HostFuncFailed) instead of passing null
  uint32_t xref_in(uint128_t v, bool *full) {
    const uint64_t x = uint64_t(v);
    if (x < 0x80000000ull || x == 0xFFFFFFFFull) return uint32_t(x);
    std::lock_guard<std::mutex> g(xref_mu);
    auto it = xref_ids.find(x);
    if (it != xref_ids.end()) return it->second;
    if (xref_vals.size() >= 0x7FFFFFFFull) {   // (2^31 - 1 distinct values)
      *full = true;
      return 0xFFFFFFFFu;
    }
    const uint32_t h = 0x80000000u + uint32_t(xref_vals.size());
    xref_vals.push_back(x);
    xref_ids.emplace(x, h);
    return h;
  }
  uint128_t xref_out(uint32_t h) {
    if (h < 0x80000000u || h == 0xFFFFFFFFu) return h;
    std::lock_guard<std::mutex> g(xref_mu);
    return h - 0x80000000u < xref_vals.size() ? xref_vals[h - 0x80000000u] : h;
  }
  uint8_t fail(uint8_t code, const std::string &m) {
    last_error = m;
    return code;
  }
  bool hip_ok(hipError_t e, const char *what) {
    if (e == hipSuccess) return true;
    last_error = std::string(what) + ": " + hipGetErrorString(e);
    return false;
  }
  // wait for queued Reset kernels before a host copy touches instance state
  bool settle() {
    if (reset_deferred && !wbh_reset_now(this)) return false;
    if (!reset_pending) return true;
    reset_pending = false;
    return hip_ok(hipStreamSynchronize(stream), "reset kernels");
  }
};

namespace wbh {

// The context's device current on the calling thread for a call's span (restored after):
// a multi-device batch drives each shard from its own thread, and a caller may have any
// device current.
struct DevScope {
  int prev = -1;
  explicit DevScope(const WasmEdge_BatchContext *C) {
    int cur = -1;
    if (C && C->stream && hipGetDevice(&cur) == hipSuccess && cur != C->device &&
        hipSetDevice(C->device) == hipSuccess)
      prev = cur;
  }
  ~DevScope() { if (prev >= 0) (void)hipSetDevice(prev); }
  DevScope(const DevScope &) = delete;
  DevScope &operator=(const DevScope &) = delete;
};

// multi.cpp: the placement of instance ids over shards, and the routed API
bool placement(uint32_t n, uint32_t g_count, uint32_t part, uint32_t inst, uint32_t *g, uint32_t *local);
uint32_t shard_size(uint32_t n, uint32_t g_count, uint32_t part, uint32_t g);

constexpr uint32_t kBlockWords = 1024;   // host-view block: 4 KiB of each of a wave's 64 lanes

// Word `w` of lane `lane` within its wave's memory region, granules of 2^g words
// (dbc_ops.h GMem): ((w >> g) * 64 + lane) * 2^g + (w & (2^g - 1)).
inline size_t lane_word(uint64_t w, uint32_t lane, uint32_t g) {
  return (size_t(w >> g) << (6 + g)) + (size_t(lane) << g) + size_t(w & ((1u << g) - 1u));
}

// One service round's copy of linear-memory rows across all parked waves (hostcall.cpp):
// row b = words [64b, 64b + 64) of every lane, 16 KiB per wave, contiguous on the device
// in each wave's region; the first touch by ANY wave fetches the row of every wave with
// one 2D copy, and a dirty row goes back with one 2D copy. Host functions of a SIMT batch
// touch the same few addresses in every instance, so a round moves a few rows, not 64K
// small pieces. Past a byte budget a row is left to the per-wave blocks of WaveView.
struct RoundCache {
  static constexpr uint32_t kRowWords = 64;
  WasmEdge_BatchContext *C = nullptr;
  uint32_t w0 = 0, nw = 0;             // waves [w0, w0 + nw)
  size_t budget = size_t(1) << 30;     // host bytes for rows
  struct Row {
    std::once_flag once;
    bool cached = false, ok = true;
    std::atomic<bool> dirty{false};
    std::vector<uint32_t> w;           // [nw][64 lanes * kRowWords]
  };
  std::mutex mu;
  std::unordered_map<uint32_t, std::unique_ptr<Row>> rows;
  std::atomic<size_t> used{0};
  // the wave's part of row b (4096 words, lane-interleaved), or nullptr (not cached)
  uint32_t *get(uint32_t b, uint32_t wave, bool *fail);
  void mark_dirty(uint32_t b);
  bool flush();
};

// The host's view of one wave's linear memories during a host-call service round
// (hostcall.cpp): through the round's RoundCache when it holds the row, else blocks of
// kBlockWords rows (256 KiB, contiguous on the device) fetched on first touch and written
// back once at the end of the wave; the lanes' page counts and write marks come from one
// copy of the instance state per round.
struct WaveView {
  RoundCache *rc = nullptr;
  struct RowRef { uint32_t b; uint32_t *p; bool dirty; };
  std::vector<RowRef> rows;          // this wave's rows of rc, looked up once each
  WasmEdge_BatchContext *C = nullptr;
  uint32_t wave = 0;
  const uint32_t *pages = nullptr;   // [64]
  uint32_t *hwm = nullptr;           // [64], raised by writes
  bool hwm_dirty = false, ok = true;
  struct Block { std::vector<uint32_t> w; bool dirty = false; };
  std::vector<std::pair<uint32_t, Block>> blocks;
  Block *block(uint32_t b);
  // bytes [off, off+len) of `lane`; 0 or MemoryOutOfBounds (0x88) / RuntimeError
  uint8_t rw(uint32_t lane, uint32_t off, uint32_t len, uint8_t *dst, const uint8_t *src);
  bool flush();
};

uint8_t mem_rw(WasmEdge_BatchContext *C, uint32_t Inst, uint32_t Off, uint32_t Len,
               uint8_t *Dst, const uint8_t *Src);
// pool rows (hostcall.cpp): give wave `wave` rows up to `rows` pool pages (false: no
// device memory for all of them; it keeps what it got); return every row at Reset
bool pool_reserve(WasmEdge_BatchContext *C, uint32_t wave, uint32_t rows);
bool pool_reset(WasmEdge_BatchContext *C);
// the call stack grown to hold `need` cells per lane (at least twice its size; between
// launches, its contents copied); false: no device memory for it (the caller then stops
// growing it: calls past it trap 0xB0 as with a fixed CallStackCells)
bool grow_stack(WasmEdge_BatchContext *C, uint64_t need);
bool shrink_stack(WasmEdge_BatchContext *C);
// grow the reserved layout to at least `need` pages per instance (up to `want`), within the
// device memory and MemoryPoolBytes; live: keep the instances' memory (pool rows move into
// the layout), else the next Reset rewrites it (mem_fresh). false only on a device error;
// a layout that cannot grow stays as it was (true)
bool grow_layout(WasmEdge_BatchContext *C, uint32_t need, uint32_t want, bool live);
bool pool_upload(WasmEdge_BatchContext *C);
int64_t service_host_calls(WasmEdge_BatchContext *C);
uint64_t mem_size(const WasmEdge_BatchMemoryContext *M);   // bytes of the instance's memory

}  // namespace wbh
