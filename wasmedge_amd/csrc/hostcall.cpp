// hostcall.cpp -- the host side of the import yield path: lanes parked
// at a host import are served on the CPU between kernel launches, the batched form of the
// reference's host-function call (lib/executor/helper.cpp:35-97, hostfunc.h:25-40).
//
// A service round moves data in bulk, never per lane:
//   * status, the import index (hcall) and the staged arguments (hbuf) of every lane:
//     one copy each;
//   * the page counts and write marks of every lane: one strided copy each (one 256-byte
//     row per wave);
//   * linear memory: a host function's reads and writes go through the round's
//     RoundCache: the first touch of a 256-byte row by any lane fetches that row of every
//     parked wave with one 2D copy (16 KiB per wave, contiguous in the lane-interleaved
//     layout), and dirty rows go back with one 2D copy each. 64K lanes calling fd_write
//     thus cost a handful of copies. Past the cache's byte budget (a host function that
//     reads a lot of memory) a wave's WaveView fetches 256 KiB per-wave blocks instead.
// Waves are served by a pool of host threads (a wave's lanes and blocks belong to one
// thread), so host functions must be reentrant, as the reference's are under its
// concurrent VM::execute (include/vm/vm.h:137-141).
#include <algorithm>
#include <atomic>
#include <thread>

#include "batch_ctx.h"

namespace wbh {

void RoundCache::mark_dirty(uint32_t b) {
  std::lock_guard<std::mutex> lock(mu);
  rows[b]->dirty = true;
}

uint32_t *RoundCache::get(uint32_t b, uint32_t wave, bool *fail) {
  if (wave < w0 || wave >= w0 + nw) return nullptr;
  // pool pages sit at a different address per wave: left to the per-wave blocks
  if (uint64_t(b + 1) * kRowWords > C->mem_words) return nullptr;
  Row *r;
  {
    std::lock_guard<std::mutex> lock(mu);
    auto &slot = rows[b];
    if (!slot) slot.reset(new Row);
    r = slot.get();
  }
  std::call_once(r->once, [&]() {
    const size_t row = size_t(64) * kRowWords;   // words per wave
    const size_t bytes = size_t(nw) * row * 4;
    if (used.fetch_add(bytes) + bytes > budget) return;   // left to the per-wave blocks
    r->w.resize(size_t(nw) * row);
    const size_t pitch = size_t(C->mem_words) * 64 * 4;   // one wave's memories
    const uint32_t *src = C->mem.ptr + (size_t(w0) * C->mem_words + size_t(b) * kRowWords) * 64;
    r->ok = hipMemcpy2D(r->w.data(), row * 4, src, pitch, row * 4, nw, hipMemcpyDeviceToHost) == hipSuccess;
    r->cached = true;
  });
  if (!r->cached) return nullptr;
  if (!r->ok) { *fail = true; return nullptr; }
  return r->w.data() + size_t(wave - w0) * 64 * kRowWords;
}

bool RoundCache::flush() {
  bool ok = true;
  const size_t row = size_t(64) * kRowWords, pitch = size_t(C->mem_words) * 64 * 4;
  for (auto &e : rows) {
    Row &r = *e.second;
    if (!r.cached || !r.ok || !r.dirty) continue;
    uint32_t *dst = C->mem.ptr + (size_t(w0) * C->mem_words + size_t(e.first) * kRowWords) * 64;
    ok &= hipMemcpy2D(dst, pitch, r.w.data(), row * 4, row * 4, nw, hipMemcpyHostToDevice) == hipSuccess;
  }
  rows.clear();
  return ok;
}

WaveView::Block *WaveView::block(uint32_t b) {
  for (auto &e : blocks)
    if (e.first == b) return &e.second;
  // (a block never straddles a page: 16384 words per page, kBlockWords divides it)
  const uint32_t *src = C->wave_rows(wave, uint64_t(b) * kBlockWords);
  if (!src) { ok = false; return nullptr; }
  Block blk;
  blk.w.resize(size_t(kBlockWords) * 64);
  if (hipMemcpy(blk.w.data(), src, blk.w.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) {
    ok = false;
    return nullptr;
  }
  blocks.emplace_back(b, std::move(blk));
  return &blocks.back().second;
}

uint8_t WaveView::rw(uint32_t lane, uint32_t off, uint32_t len, uint8_t *dst, const uint8_t *src) {
  const uint64_t end = uint64_t(off) + len;
  if (end > (uint64_t(pages[lane]) << 16)) return kMemoryOutOfBounds;   // memory.h:74-78
  uint64_t a = off;
  while (a < end) {
    const uint32_t w = uint32_t(a >> 2);
    if (rc) {   // the round's rows first
      bool fail = false;
      const uint32_t rb = w / RoundCache::kRowWords;
      RowRef *ref = nullptr;
      for (auto &x : rows)
        if (x.b == rb) { ref = &x; break; }
      if (!ref) {
        rows.push_back(RowRef{rb, rc->get(rb, wave, &fail), false});
        ref = &rows.back();
      }
      if (uint32_t *row = ref->p) {
        if (src && !ref->dirty) { rc->mark_dirty(rb); ref->dirty = true; }
        const uint64_t rend = std::min<uint64_t>(end, uint64_t(rb + 1) * RoundCache::kRowWords * 4);
        for (; a < rend; a++) {
          uint32_t &word = row[lane_word((a >> 2) % RoundCache::kRowWords, lane, C->mlog)];
          const uint32_t sh = 8 * uint32_t(a & 3);
          if (dst) *dst++ = uint8_t(word >> sh);
          else word = (word & ~(0xFFu << sh)) | (uint32_t(*src++) << sh);
        }
        continue;
      }
      if (fail) return kRuntimeError;
    }
    const uint32_t b = w / kBlockWords;
    Block *blk = block(b);
    if (!blk) return kRuntimeError;
    // bytes of this block: up to the block's last word
    const uint64_t bend = std::min<uint64_t>(end, uint64_t(b + 1) * kBlockWords * 4);
    for (; a < bend; a++) {
      uint32_t &word = blk->w[lane_word((a >> 2) % kBlockWords, lane, C->mlog)];
      const uint32_t sh = 8 * uint32_t(a & 3);
      if (dst) *dst++ = uint8_t(word >> sh);
      else word = (word & ~(0xFFu << sh)) | (uint32_t(*src++) << sh);
    }
    if (src) blk->dirty = true;
  }
  if (src && len && end > hwm[lane]) {   // raise the write mark: Reset re-inits these bytes
    hwm[lane] = end > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(end);
    hwm_dirty = true;
  }
  return 0;
}

bool WaveView::flush() {
  for (auto &e : blocks) {
    if (!e.second.dirty) continue;
    uint32_t *dst = C->wave_rows(wave, uint64_t(e.first) * kBlockWords);
    if (!dst || hipMemcpy(dst, e.second.w.data(), e.second.w.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
      ok = false;
  }
  blocks.clear();
  return ok;
}

uint64_t mem_size(const WasmEdge_BatchMemoryContext *M) {
  if (M->view) return uint64_t(M->view->pages[M->inst % 64]) << 16;
  return uint64_t(WasmEdge_BatchGetMemoryPages(M->ctx, M->inst)) << 16;
}

// Read (dst) or write (src) bytes of one instance's linear memory outside a service round
// (WasmEdge_BatchGetMemory/SetMemory): a one-lane WaveView over its wave's blocks.
uint8_t mem_rw(WasmEdge_BatchContext *C, uint32_t Inst, uint32_t Off, uint32_t Len,
               uint8_t *Dst, const uint8_t *Src) {
  if (Inst >= C->n) return C->fail(kRuntimeError, "instance index out of range");
  if (!C->settle()) return kRuntimeError;
  const uint32_t lane = Inst % 64;
  uint32_t pages[64] = {0}, hwm[64] = {0};
  pages[lane] = WasmEdge_BatchGetMemoryPages(C, Inst);
  if (uint64_t(Off) + Len > (uint64_t(pages[lane]) << 16)) return kMemoryOutOfBounds;   // memory.h:74-78
  if (Len == 0) return 0;
  uint32_t *mark = C->lstate.ptr + (size_t(Inst / 64) * C->ls_slots + LS_HWM) * 64 + lane;
  if (Src && !C->hip_ok(hipMemcpy(&hwm[lane], mark, 4, hipMemcpyDeviceToHost), "memory"))
    return kRuntimeError;
  WaveView view;
  view.C = C;
  view.wave = Inst / 64;
  view.pages = pages;
  view.hwm = hwm;
  const uint8_t e = view.rw(lane, Off, Len, Dst, Src);
  if (!view.flush()) { C->last_error = "memory: device copy failed"; return kRuntimeError; }
  if (e) return e;
  // the raised write mark (LS_HWM): the next Reset re-initialises these bytes
  if (view.hwm_dirty && !C->hip_ok(hipMemcpy(mark, &hwm[lane], 4, hipMemcpyHostToDevice), "memory"))
    return kRuntimeError;
  return 0;
}

// ---- pool rows for pages past the reserved layout ------------------------------------
// A row = one pool page of a wave: 64 lanes x 64 KiB, interleaved like the reserved layout.
constexpr size_t kRowBytes = size_t(64) << 16;

// One more chunk of zeroed rows: at least `want` rows, growing with the pool (1/4 of what
// it holds, at most 1 GiB at a time) so that few hipMallocs serve a growing batch; falls
// back to exactly `want` when the larger chunk does not fit, and respects MemoryPoolBytes.
static bool pool_chunk(WasmEdge_BatchContext *C, size_t want) {
  size_t rows = std::max<size_t>(want, std::min<size_t>(256, std::max<size_t>(16, C->pool_bytes / kRowBytes / 4)));
  const size_t cap = C->conf.MemoryPoolBytes;
  if (cap) {   // within the cap: what is left of it, if that covers `want`
    // (the reserved layout's growth past its initial size counts too: grow_layout)
    const size_t used = C->pool_bytes + size_t(C->rpages - C->rpages0) * C->nwaves * kRowBytes;
    const size_t left = used < cap ? (cap - used) / kRowBytes : 0;
    if (left < want) return false;
    rows = std::min(rows, left);
  }
  for (int attempt = 0; attempt < 2; attempt++, rows = want) {
    void *p = nullptr;
    if (hipMalloc(&p, rows * kRowBytes) != hipSuccess) { (void)hipGetLastError(); continue; }
    if (hipMemset(p, 0, rows * kRowBytes) != hipSuccess) { (void)hipFree(p); return false; }
    C->pool_chunks.emplace_back(p, rows * kRowBytes);
    C->pool_bytes += rows * kRowBytes;
    for (size_t r = rows; r-- > 0;)
      C->pool_free.push_back(reinterpret_cast<uint64_t>(p) + r * kRowBytes);
    return true;
  }
  return false;
}

bool pool_reserve(WasmEdge_BatchContext *C, uint32_t wave, uint32_t rows) {
  uint32_t &have = C->pt_n[wave];
  if (rows <= have) return true;
  if (rows > C->pt_w) {   // widen the page table (every wave's row of it)
    uint32_t w = std::max<uint32_t>(rows, std::max<uint32_t>(16, C->pt_w * 2));
    w = std::min<uint32_t>(w, C->mem_max_pages - C->rpages);
    // the new device table first: when it cannot be had, the old table, its width and its
    // device copy stay as they were and the grow yields -1 (Allocator::resize failing)
    wbh::DevBuf<uint64_t> nt;
    if (!nt.alloc(size_t(C->nwaves) * w)) {
      (void)hipGetLastError();
      return false;
    }
    std::vector<uint64_t> t(size_t(C->nwaves) * w, 0);
    for (uint32_t v = 0; v < C->nwaves; v++)
      for (uint32_t k = 0; k < C->pt_n[v]; k++) t[size_t(v) * w + k] = C->pt_host[size_t(v) * C->pt_w + k];
    C->pt_host.swap(t);
    C->pt_w = w;
    std::swap(C->ptab.ptr, nt.ptr);
    std::swap(C->ptab.n, nt.n);   // (nt frees the old table)
    C->pt_dirty = true;
  }
  while (have < rows) {
    if (C->pool_free.empty() && !pool_chunk(C, rows - have)) return false;
    C->pt_host[size_t(wave) * C->pt_w + have++] = C->pool_free.back();
    C->pool_free.pop_back();
    C->pool_used = C->pt_dirty = true;
  }
  return true;
}

bool pool_upload(WasmEdge_BatchContext *C) {
  if (!C->pt_dirty) return true;
  C->pt_dirty = false;
  return C->hip_ok(hipMemcpy(C->ptab.ptr, C->pt_host.data(), C->pt_host.size() * 8, hipMemcpyHostToDevice),
                   "page table");
}

// Reset (a fresh instantiation): every row back to the free list, zeroed again.
bool pool_reset(WasmEdge_BatchContext *C) {
  if (!C->pool_used) return true;
  C->pool_used = false;
  C->pool_free.clear();
  for (const auto &ch : C->pool_chunks) {
    if (!C->hip_ok(hipMemsetAsync(ch.first, 0, ch.second, C->stream), "pool reset")) return false;
    for (size_t r = ch.second / kRowBytes; r-- > 0;)
      C->pool_free.push_back(reinterpret_cast<uint64_t>(ch.first) + r * kRowBytes);
  }
  std::fill(C->pt_host.begin(), C->pt_host.end(), 0ull);
  std::fill(C->pt_n.begin(), C->pt_n.end(), 0u);
  C->pt_dirty = true;
  if (!C->pt_host.empty() &&
      !C->hip_ok(hipMemsetAsync(C->ptab.ptr, 0, C->pt_host.size() * 8, C->stream), "page table"))
    return false;
  C->pt_dirty = false;
  return true;
}

// The reserved layout grown (DESIGN.md "Paged growth"): every page below the new rpages in
// the lane-interleaved layout, where every engine -- compiled runs, threaded core, compiled
// step -- addresses it directly, instead of pool rows that only the per-lane step reaches
// through the page table. Grown between launches, when no lane runs: in a service round
// (live: the old layout's rows and the pool rows are copied to their places in the new one,
// device to device) or at a Reset (which rewrites every page anyway). Bounded by 3/4 of the
// device memory this context holds or could get, and by MemoryPoolBytes past the initial
// layout; WB_RELAYOUT=0 keeps the layout fixed (A/B aid). Results never depend on it.
bool grow_layout(WasmEdge_BatchContext *C, uint32_t need, uint32_t want, bool live) {
  if (const char *e = getenv("WB_RELAYOUT"))
    if (e[0] == '0') return true;
  need = std::min(need, C->mem_max_pages);
  want = std::min(std::max(want, need), C->mem_max_pages);
  if (need <= C->rpages) return true;
  const uint64_t wave_page = uint64_t(64) << 16;   // one page of a wave's 64 lanes
  const uint64_t per_page = uint64_t(C->nwaves) * wave_page;
  size_t free_b = 0, total_b = 0;
  (void)hipMemGetInfo(&free_b, &total_b);
  // (live: the old layout and the pool stay until their rows are copied)
  const uint64_t held = live ? 0 : uint64_t(C->rpages) * per_page + C->pool_bytes;
  uint64_t cap = (uint64_t(free_b) + held) / 4 * 3 / per_page;
  if (C->conf.MemoryPoolBytes) cap = std::min<uint64_t>(cap, C->rpages0 + C->conf.MemoryPoolBytes / per_page);
  if (cap < need) return true;
  const uint32_t target = uint32_t(std::min<uint64_t>(want, cap));
  const size_t old_words = C->mem_words, new_words = size_t(target) << 14;
  if (!live) {   // (the next Reset writes every page: nothing is copied)
    // the new layout is allocated before the old one goes, so a failure leaves the context
    // with the layout it had (never without one); the pool rows go first only when the
    // new layout does not fit beside them
    const size_t bytes = (size_t(C->nwaves) * new_words * 64 + 64) * 4;
    uint32_t *nm = nullptr;
    auto drop_pool = [&] {
      for (const auto &ch : C->pool_chunks) (void)hipFree(ch.first);
      C->pool_chunks.clear();
      C->pool_free.clear();
      C->pool_bytes = 0;
    };
    if (hipMalloc(&nm, bytes) != hipSuccess) {
      (void)hipGetLastError();
      drop_pool();
      if (hipMalloc(&nm, bytes) != hipSuccess) {
        (void)hipGetLastError();   // (no room after all: the layout it had)
        C->pool_used = true;   // (its pool rows went: pool_reset restarts the table)
        return true;
      }
    }
    drop_pool();
    (void)hipFree(C->mem.ptr);
    C->mem.ptr = nm;
    C->mem.n = size_t(C->nwaves) * new_words * 64 + 64;
    C->mem_fresh = true;
  } else {
    uint32_t *nm = nullptr;
    if (hipMalloc(&nm, (size_t(C->nwaves) * new_words * 64 + 64) * 4) != hipSuccess) {
      (void)hipGetLastError();
      return true;
    }
    hipStream_t s = C->stream;
    bool ok = hipMemsetAsync(nm, 0, (size_t(C->nwaves) * new_words * 64 + 64) * 4, s) == hipSuccess;
    // each wave's rows of the old layout (one 2D copy while its pitches allow), then its
    // pool rows as the pages after them
    const bool one = new_words * 256 < (size_t(1) << 31);
    if (ok && one)
      ok = hipMemcpy2DAsync(nm, new_words * 256, C->mem.ptr, old_words * 256, old_words * 256, C->nwaves,
                            hipMemcpyDeviceToDevice, s) == hipSuccess;
    for (uint32_t w = 0; ok && w < C->nwaves; w++) {
      if (!one)
        ok = hipMemcpyAsync(nm + size_t(w) * new_words * 64, C->mem.ptr + size_t(w) * old_words * 64, old_words * 256,
                            hipMemcpyDeviceToDevice, s) == hipSuccess;
      for (uint32_t k = 0; ok && k < C->pt_n[w] && C->rpages + k < target; k++)
        ok = hipMemcpyAsync(nm + (size_t(w) * new_words + (size_t(C->rpages + k) << 14)) * 64,
                            reinterpret_cast<const void *>(C->pt_host[size_t(w) * C->pt_w + k]),
                            size_t(1) << 22, hipMemcpyDeviceToDevice, s) == hipSuccess;
    }
    if (!ok || hipStreamSynchronize(s) != hipSuccess) {
      (void)hipFree(nm);
      return C->hip_ok(hipGetLastError(), "memory layout copy");
    }
    (void)hipFree(C->mem.ptr);
    C->mem.ptr = nm;
    C->mem.n = size_t(C->nwaves) * new_words * 64 + 64;
    // pool rows past the new layout (none when it covers every page the lanes hold) stay
    const uint32_t moved = target - C->rpages;
    bool any_left = false;
    for (uint32_t w = 0; w < C->nwaves; w++) {
      const uint32_t have = C->pt_n[w], keep = have > moved ? have - moved : 0;
      for (uint32_t k = 0; k < keep; k++)
        C->pt_host[size_t(w) * C->pt_w + k] = C->pt_host[size_t(w) * C->pt_w + moved + k];
      for (uint32_t k = keep; k < have; k++) C->pt_host[size_t(w) * C->pt_w + k] = 0;
      C->pt_n[w] = keep;
      any_left |= keep != 0;
    }
    if (!any_left) {   // every row moved: the pool goes
      for (const auto &ch : C->pool_chunks) (void)hipFree(ch.first);
      C->pool_chunks.clear();
      C->pool_free.clear();
      C->pool_bytes = 0;
      C->pool_used = false;
    }
    C->pt_dirty = true;
  }
  if (!C->pt_host.empty() && C->pool_bytes == 0) {
    std::fill(C->pt_host.begin(), C->pt_host.end(), 0ull);
    std::fill(C->pt_n.begin(), C->pt_n.end(), 0u);
    C->pt_dirty = true;
  }
  C->rpages = target;
  C->mem_words = uint32_t(new_words);
  C->grow_host = C->mem_max_pages > target;
  if (!live) C->pool_used = false;
  return pool_upload(C);
}

// The call stack's HBM part doubled (at least), between launches: [wave][slot][64] at the
// old depth copied into the new one (one 2D copy while its pitch allows), the old freed.
// Bounded by CallStackMaxBytes (0: an eighth of the device's memory) and by 3/4 of the
// device memory left, so a runaway recursion cannot take the device from the context's
// own memory growth or from other contexts; false when that does not hold `need` cells.
// BatchReset gives the growth back (shrink_stack).
bool grow_stack(WasmEdge_BatchContext *C, uint64_t need) {
  const uint64_t old_d = C->gs_depth;
  uint64_t d = std::max<uint64_t>(old_d * 2, need);
  size_t free_b = 0, total_b = 0;
  (void)hipMemGetInfo(&free_b, &total_b);
  const uint64_t per_cell = uint64_t(C->nwaves) * 256;   // one cell of every lane
  const uint64_t share = C->conf.CallStackMaxBytes ? C->conf.CallStackMaxBytes : uint64_t(total_b) / 8;
  const uint64_t held = old_d * per_cell;                // (freed once the copy is made)
  uint64_t cap = std::min<uint64_t>(uint64_t(free_b) / 4 * 3 / per_cell, 0x7FFFFFFFull / 256);
  cap = std::min<uint64_t>(cap, std::max<uint64_t>(share, held) / per_cell);
  d = std::min(d, cap);
  if (d <= old_d || d < need) return false;
  uint32_t *ns = nullptr;
  if (hipMalloc(&ns, size_t(C->nwaves) * d * 256) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  bool ok = hipMemcpy2DAsync(ns, d * 256, C->gstack.ptr, old_d * 256, old_d * 256, C->nwaves,
                             hipMemcpyDeviceToDevice, C->stream) == hipSuccess &&
            hipStreamSynchronize(C->stream) == hipSuccess;
  if (!ok) {
    (void)hipFree(ns);
    (void)hipGetLastError();
    return false;
  }
  (void)hipFree(C->gstack.ptr);
  C->gstack.ptr = ns;
  C->gstack.n = size_t(C->nwaves) * d * 64;
  C->gs_depth = uint32_t(d);
  return true;
}

// At BatchReset: the call stack back to its first depth and growth re-armed (a stack that
// once hit its bound grows again for the next run). Between launches; the stack's contents
// are dead after a Reset.
bool shrink_stack(WasmEdge_BatchContext *C) {
  C->gs_grow = C->gs_grow0;
  if (C->gs_depth <= C->gs_depth0) return true;
  uint32_t *ns = nullptr;
  if (!C->hip_ok(hipStreamSynchronize(C->stream), "call stack")) return false;
  if (hipMalloc(&ns, size_t(C->nwaves) * C->gs_depth0 * 256) != hipSuccess) {
    (void)hipGetLastError();
    return true;   // (keeps the deeper stack it has)
  }
  (void)hipFree(C->gstack.ptr);
  C->gstack.ptr = ns;
  C->gstack.n = size_t(C->nwaves) * C->gs_depth0 * 64;
  C->gs_depth = C->gs_depth0;
  return true;
}

// Every lane's per-lane tables relaid out wider, between launches: table t to at least
// need[t] entries (at least double, within table_widen_limit), the others as they were.
// [wave][tab_words][64] copied table by table into a new buffer whose new slots are null;
// the image Reset starts from and tabinfo follow. False (nothing changed) when 3/4 of the
// device memory left does not hold the new tables.
static bool widen_tables(WasmEdge_BatchContext *C, const std::vector<uint64_t> &need) {
  wb::Program &P = C->prog;
  std::vector<uint32_t> info(P.tabinfo.size());
  uint64_t words = 0;
  for (uint32_t t = 0; t < P.ntables; t++) {
    uint64_t cap = P.tabinfo[2 * t + 1];
    if (need[t] > cap)
      cap = std::min<uint64_t>(wb::table_widen_limit(P.tables[t]), std::max<uint64_t>(need[t], 2 * cap));
    info[2 * t] = uint32_t(words);
    info[2 * t + 1] = uint32_t(cap);
    words += cap;
  }
  size_t free_b = 0, total_b = 0;
  (void)hipMemGetInfo(&free_b, &total_b);
  const uint64_t nw = C->nwaves, bytes = nw * words * 256;
  if (words >= (1ull << 28) || bytes > uint64_t(free_b) / 4 * 3) return false;
  uint32_t *nt = nullptr;
  if (hipMalloc(&nt, bytes) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  bool ok = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(nt), 0xFFFFFFFFu, nw * words * 64, C->stream) == hipSuccess;
  for (uint32_t t = 0; ok && t < P.ntables; t++) {
    const uint64_t f = P.tabinfo[2 * t], c = P.tabinfo[2 * t + 1], nf = info[2 * t];
    if (!c) continue;
    // (one 2D copy per table: rows = waves, each the table's c x 64 words of that wave)
    ok = hipMemcpy2DAsync(nt + nf * 64, words * 256, C->ltab.ptr + f * 64, uint64_t(P.tab_words) * 256,
                          c * 256, nw, hipMemcpyDeviceToDevice, C->stream) == hipSuccess;
  }
  ok = ok && hipStreamSynchronize(C->stream) == hipSuccess;
  if (!ok) {
    (void)hipFree(nt);
    (void)hipGetLastError();
    return false;
  }
  std::vector<uint32_t> img(words, 0xFFFFFFFFu);
  for (uint32_t t = 0; t < P.ntables; t++)
    std::copy(P.tab_image.begin() + P.tabinfo[2 * t], P.tab_image.begin() + P.tabinfo[2 * t] + P.tabinfo[2 * t + 1],
              img.begin() + info[2 * t]);
  (void)hipFree(C->ltab.ptr);
  C->ltab.ptr = nt;
  C->ltab.n = nw * words * 64;
  P.tab_image.swap(img);
  P.tabinfo.swap(info);
  P.tab_words = uint32_t(words);
  return C->tab_image.upload(P.tab_image, C->stream) && C->tabinfo.upload(P.tabinfo, C->stream) &&
         hipStreamSynchronize(C->stream) == hipSuccess;
}

// Lanes parked at a table.grow past their table's capacity (WB_TGROW_CALL | t; the request
// n in their staged cell): every table asked for widens to the largest size a lane asks
// (widen_tables), and every such lane runs its grow again -- or, with no device memory left
// for it, the tables stop widening and the grow returns -1 as at a fixed capacity.
static bool serve_table_grows(WasmEdge_BatchContext *C, const std::vector<uint32_t> &parked,
                              std::vector<uint32_t> &hcall, const std::vector<uint32_t> &hbuf,
                              int64_t *resumed) {
  const wb::Program &P = C->prog;
  const uint32_t nw = C->nwaves, hb = C->hb_cells;
  std::vector<uint8_t> asked(P.ntables, 0);
  bool any = false;
  for (uint32_t i : parked)
    if ((hcall[i] & WB_TGROW_MASK) == WB_TGROW_CALL) {
      asked[hcall[i] & ~WB_TGROW_MASK] = 1;
      any = true;
    }
  if (!any) return true;
  // table sizes of the tables asked for: one 256-byte row per wave each
  const size_t row = 64 * sizeof(uint32_t), pitch = size_t(C->ls_slots) * row;
  std::vector<std::vector<uint32_t>> size(P.ntables);
  for (uint32_t t = 0; t < P.ntables; t++) {
    if (!asked[t]) continue;
    size[t].assign(size_t(nw) * 64, 0);
    if (!C->hip_ok(hipMemcpy2D(size[t].data(), row, C->lstate.ptr + size_t(LS_GLOBALS + P.global_cells + t) * 64,
                               pitch, row, nw, hipMemcpyDeviceToHost), "table sizes"))
      return false;
  }
  std::vector<uint64_t> need(P.ntables, 0);
  for (uint32_t i : parked)
    if ((hcall[i] & WB_TGROW_MASK) == WB_TGROW_CALL) {
      const uint32_t t = hcall[i] & ~WB_TGROW_MASK;
      need[t] = std::max<uint64_t>(need[t], uint64_t(size[t][i]) + hbuf[size_t(i) * hb]);
    }
  if (!widen_tables(C, need)) C->tg_grow = false;
  for (uint32_t i : parked)
    if ((hcall[i] & WB_TGROW_MASK) == WB_TGROW_CALL) {
      hcall[i] = 0;   // (no result cells: the grow runs again)
      ++*resumed;
    }
  return true;
}

// Lanes parked at a memory.grow past their wave's rows (WB_GROW_CALL; the request n in
// their staged result cell): per wave, rows for the largest request (plus a quarter of what
// the wave holds, so that a lane growing page by page parks rarely), then each lane's grow
// completes -- old size, pages raised -- or returns -1 when the device has no memory for
// its pages (growPage failing in Allocator::resize, memory.h:104-109).
static void serve_grows(WasmEdge_BatchContext *C, const std::vector<uint32_t> &parked,
                        std::vector<uint32_t> &hcall, std::vector<uint32_t> &hbuf,
                        std::vector<uint32_t> &pages, bool *pages_dirty, int64_t *resumed) {
  const uint32_t hb = C->hb_cells;
  // first the reserved layout grows to take every request (with a quarter of slack, so a
  // lane growing page by page rarely parks again): the grown pages then run on every engine
  uint32_t top = 0;
  for (uint32_t i : parked)
    if (hcall[i] == WB_GROW_CALL) top = std::max(top, pages[i] + hbuf[size_t(i) * hb]);
  for (uint32_t w = 0; w < C->nwaves; w++) top = std::max(top, C->rpages + C->pt_n[w]);
  if (top > C->rpages)
    (void)grow_layout(C, top, top + std::max<uint32_t>(4, top / 4), true);
  const uint32_t R = C->rpages;
  // per wave, the lanes' requests smallest first: when the device runs out, the lanes
  // that need fewer pages still get them
  std::vector<std::pair<uint32_t, uint32_t>> need;   // (wave, rows)
  for (uint32_t i : parked)
    if (hcall[i] == WB_GROW_CALL && pages[i] + hbuf[size_t(i) * hb] > R)
      need.emplace_back(i / 64, pages[i] + hbuf[size_t(i) * hb] - R);
  std::sort(need.begin(), need.end());
  const uint32_t room = C->mem_max_pages - R;
  for (size_t k = 0; k < need.size(); k++) {
    const uint32_t w = need[k].first, rows = need[k].second;
    if (rows <= C->pt_n[w]) continue;
    if (k > 0 && need[k - 1].first == w && need[k - 1].second > C->pt_n[w]) continue;   // failed
    const uint32_t slack = std::min<uint32_t>(room, std::max(rows, C->pt_n[w] + std::max<uint32_t>(4, C->pt_n[w] / 4)));
    if (!pool_reserve(C, w, slack)) (void)pool_reserve(C, w, rows);
  }
  for (uint32_t i : parked) {
    if (hcall[i] != WB_GROW_CALL) continue;
    const uint32_t n = hbuf[size_t(i) * hb];
    uint32_t &res = hbuf[size_t(i) * hb];
    if (pages[i] + n <= R || pages[i] + n - R <= C->pt_n[i / 64]) {
      res = pages[i];
      pages[i] += n;
      *pages_dirty = true;
    } else {
      res = 0xFFFFFFFFu;
    }
    hcall[i] = 1;   // one result cell
    ++*resumed;
  }
}

// Serve every lane parked at a host import: call its host function with the args the
// kernel staged in hbuf, stage the results (or end the lane with the host's ErrCode;
// Terminated 0x01 ends it too, engine.cpp:62-64). Returns the number of lanes to resume,
// or -1 on a device error.
int64_t service_host_calls(WasmEdge_BatchContext *C) {
  // the shards of a multi-device batch serve their rounds one at a time unless the caller
  // declared its host functions reentrant (HostThreads > 1)
  std::unique_lock<std::mutex> shard_lock;
  if (C->host_mu) shard_lock = std::unique_lock<std::mutex>(*C->host_mu);
  const wb::Program &P = C->prog;
  const uint32_t n = C->n, hb = C->hb_cells, nw = C->nwaves;
  std::vector<uint8_t> st(n);
  if (!C->hip_ok(hipMemcpy(st.data(), C->status.ptr, n, hipMemcpyDeviceToHost), "status"))
    return -1;
  // parked lanes grouped by wave: waves[k] = (wave, first index into `parked`)
  std::vector<uint32_t> parked;
  std::vector<std::pair<uint32_t, uint32_t>> waves;
  for (uint32_t i = 0; i < n; i++)
    if (st[i] == WB_ERR_HOST_CALL) {
      if (waves.empty() || waves.back().first != i / 64) waves.emplace_back(i / 64, uint32_t(parked.size()));
      parked.push_back(i);
    }
  if (parked.empty()) return 0;
  waves.emplace_back(nw, uint32_t(parked.size()));   // sentinel
  std::vector<uint32_t> hcall(n), hbuf(size_t(n) * hb);
  if (!C->hip_ok(hipMemcpy(hcall.data(), C->hcall.ptr, size_t(n) * 4, hipMemcpyDeviceToHost), "hcall") ||
      !C->hip_ok(hipMemcpy(hbuf.data(), C->hbuf.ptr, hbuf.size() * 4, hipMemcpyDeviceToHost), "hbuf"))
    return -1;
  // page counts and write marks: one 256-byte row per wave each
  const size_t row = 64 * sizeof(uint32_t), pitch = size_t(C->ls_slots) * row;
  std::vector<uint32_t> pages(size_t(nw) * 64, 0), hwm(size_t(nw) * 64, 0);
  if (P.has_mem &&
      (!C->hip_ok(hipMemcpy2D(pages.data(), row, C->lstate.ptr + LS_PAGES * 64, pitch, row, nw,
                              hipMemcpyDeviceToHost), "pages") ||
       !C->hip_ok(hipMemcpy2D(hwm.data(), row, C->lstate.ptr + LS_HWM * 64, pitch, row, nw,
                              hipMemcpyDeviceToHost), "write marks")))
    return -1;

  // gas (metered contexts): the running totals of the waves with a parked lane whose host
  // function has a cost, charged below before the function runs (helper.cpp:59-64)
  const uint64_t limit = C->conf.CostLimit;
  bool charge = false;
  if (limit)
    for (uint32_t i : parked)
      if (hcall[i] < C->hosts.size() && C->hosts[hcall[i]].fn && C->hosts[hcall[i]].cost) charge = true;
  std::vector<uint32_t> cost_lo, cost_hi;
  if (charge) {
    cost_lo.assign(size_t(nw) * 64, 0);
    cost_hi.assign(size_t(nw) * 64, 0);
    if (!C->hip_ok(hipMemcpy2D(cost_lo.data(), row, C->lstate.ptr + LS_COST * 64, pitch, row, nw,
                               hipMemcpyDeviceToHost), "costs") ||
        !C->hip_ok(hipMemcpy2D(cost_hi.data(), row, C->lstate.ptr + (LS_COST + 1) * 64, pitch, row, nw,
                               hipMemcpyDeviceToHost), "costs"))
      return -1;
  }
  // memory.grow requests first: host functions of this round then see the grown pages
  bool pages_dirty = false;
  int64_t grown = 0;
  std::vector<uint8_t> hcall_grow(parked.size(), 0);
  for (size_t j = 0; j < parked.size(); j++)
    hcall_grow[j] = hcall[parked[j]] == WB_GROW_CALL || hcall[parked[j]] == WB_STACK_CALL ||
                    (hcall[parked[j]] & WB_TGROW_MASK) == WB_TGROW_CALL;
  if (C->grow_host) {
    serve_grows(C, parked, hcall, hbuf, pages, &pages_dirty, &grown);
    if (!pool_upload(C)) return -1;
  }
  // calls past the call stack (WB_STACK_CALL): the stack doubles (or takes what the deepest
  // parked lane needs), every such lane runs its call again -- or, with no device memory
  // left for it, the stack stops growing and the call traps 0xB0 as with a fixed size
  if (C->gs_grow) {
    bool any = false;
    for (uint32_t i : parked) any |= hcall[i] == WB_STACK_CALL;
    if (any) {
      std::vector<uint32_t> gsp(size_t(nw) * 64, 0);
      if (!C->hip_ok(hipMemcpy2D(gsp.data(), row, C->lstate.ptr + LS_GSP * 64, pitch, row, nw,
                                 hipMemcpyDeviceToHost), "call stack depth"))
        return -1;
      uint64_t need = 0;
      for (uint32_t i : parked)
        if (hcall[i] == WB_STACK_CALL) need = std::max<uint64_t>(need, uint64_t(gsp[i]) + C->prog.total_cells() + 1);
      if (!grow_stack(C, need)) C->gs_grow = false;
      for (uint32_t i : parked)
        if (hcall[i] == WB_STACK_CALL) {
          hcall[i] = 0;   // (no result cells: the call runs again)
          grown++;
        }
    }
  }
  // table.grow past a table's capacity (WB_TGROW_CALL | t)
  if (C->tg_grow && !serve_table_grows(C, parked, hcall, hbuf, &grown)) return -1;
  RoundCache rc;
  rc.C = C;
  rc.w0 = waves.front().first;
  rc.nw = waves[waves.size() - 2].first - rc.w0 + 1;   // (the last entry is the sentinel)
  std::atomic<uint32_t> next{0};
  std::atomic<int64_t> resumed{0};
  std::atomic<bool> failed{false}, hwm_dirty{false};
  auto worker = [&]() {
    (void)hipSetDevice(C->device);   // the device is per host thread
    std::vector<WasmEdge_Value> args, rets;
    int64_t mine = 0;   // lanes this thread resumes (one atomic add at the end)
    for (uint32_t k; (k = next.fetch_add(1)) + 1 < waves.size();) {
      WaveView view;
      view.rc = P.has_mem ? &rc : nullptr;
      view.C = C;
      view.wave = waves[k].first;
      view.pages = &pages[size_t(view.wave) * 64];
      view.hwm = &hwm[size_t(view.wave) * 64];
      for (uint32_t j = waves[k].second; j < waves[k + 1].second; j++) {
        const uint32_t i = parked[j], f = hcall[i];
        if (hcall_grow[j]) continue;   // (memory.grow and call-stack growth: served above)
        const WasmEdge_BatchContext::HostFn h =
            f < C->hosts.size() ? C->hosts[f] : WasmEdge_BatchContext::HostFn{};
        if (!h.fn) { hcall[i] = 0xFFFFFFFFu; continue; }   // no host function: stays 0xB1
        if (charge && h.cost) {   // Stat->addCost(HostFunc.getCost()) before the call
          const uint64_t sum = (uint64_t(cost_hi[i]) << 32) | cost_lo[i], nsum = sum + h.cost;
          if (nsum > limit) {     // CostLimitExceeded: the function never runs
            st[i] = 0x03;
            hcall[i] = 0xFFFFFFFFu;
            continue;
          }
          cost_lo[i] = uint32_t(nsum);
          cost_hi[i] = uint32_t(nsum >> 32);
        }
        const wb::FuncType &t = P.types[P.funcs[f].type];
        uint32_t *cells = &hbuf[size_t(i) * hb];
        args.assign(t.params.size(), WasmEdge_Value{});
        rets.assign(t.results.size(), WasmEdge_Value{});
        uint32_t at = 0;
        for (size_t q = 0; q < t.params.size(); q++) {
          uint128_t v = 0;
          for (uint32_t c = 0; c < wb::cells_of(t.params[q]); c++) v |= uint128_t(cells[at++]) << (32 * c);
          args[q].Value = t.params[q] == wb::EXTERNREF ? C->xref_out(uint32_t(v)) : v;
          args[q].Type = static_cast<enum WasmEdge_ValType>(t.params[q]);
        }
        for (size_t q = 0; q < t.results.size(); q++)
          rets[q].Type = static_cast<enum WasmEdge_ValType>(t.results[q]);
        WasmEdge_BatchMemoryContext mc{C, i, &view};
        const WasmEdge_Result r = h.fn(h.data, &mc, args.data(), rets.data());
        if (r.Code) {            // host error or Terminated: the lane ends with that code
          st[i] = r.Code;
          hcall[i] = 0xFFFFFFFFu;
          continue;
        }
        at = 0;
        bool full = false;
        for (size_t q = 0; q < t.results.size(); q++) {
          const uint128_t v = t.results[q] == wb::EXTERNREF ? uint128_t(C->xref_in(rets[q].Value, &full)) : rets[q].Value;
          for (uint32_t c = 0; c < wb::cells_of(t.results[q]); c++) cells[at++] = uint32_t(v >> (32 * c));
        }
        if (full) {   // (the intern table is full: the host function's result cannot pass)
          st[i] = 0x8D;   // HostFuncFailed
          hcall[i] = 0xFFFFFFFFu;
          continue;
        }
        hcall[i] = at;
        mine++;
      }
      if (!view.flush()) failed = true;
      if (view.hwm_dirty) hwm_dirty = true;
    }
    resumed.fetch_add(mine);
  };
  // HostThreads 0 (the default) = one thread: host functions are called serially, as
  // before pools existed; a caller whose host functions are reentrant opts in with
  // HostThreads > 1 (a wave's lanes always stay on one thread)
  uint32_t threads = C->host_threads ? C->host_threads : 1u;
  threads = std::min<uint32_t>(threads, uint32_t(waves.size() - 1));
  if (threads <= 1) {
    worker();
  } else {
    std::vector<std::thread> pool;
    for (uint32_t t = 0; t < threads; t++) pool.emplace_back(worker);
    for (auto &th : pool) th.join();
  }
  if (!rc.flush()) failed = true;
  if (failed) { C->last_error = "host-call memory view: device copy failed"; return -1; }
  if (!C->hip_ok(hipMemcpy(C->status.ptr, st.data(), n, hipMemcpyHostToDevice), "status") ||
      !C->hip_ok(hipMemcpy(C->hcall.ptr, hcall.data(), size_t(n) * 4, hipMemcpyHostToDevice), "hcall") ||
      !C->hip_ok(hipMemcpy(C->hbuf.ptr, hbuf.data(), hbuf.size() * 4, hipMemcpyHostToDevice), "hbuf"))
    return -1;
  if (charge && (!C->hip_ok(hipMemcpy2D(C->lstate.ptr + LS_COST * 64, pitch, cost_lo.data(), row, row, nw,
                                        hipMemcpyHostToDevice), "costs") ||
                 !C->hip_ok(hipMemcpy2D(C->lstate.ptr + (LS_COST + 1) * 64, pitch, cost_hi.data(), row, row, nw,
                                        hipMemcpyHostToDevice), "costs")))
    return -1;
  if (pages_dirty && !C->hip_ok(hipMemcpy2D(C->lstate.ptr + LS_PAGES * 64, pitch, pages.data(), row, row, nw,
                                            hipMemcpyHostToDevice), "pages"))
    return -1;
  if (hwm_dirty && !C->hip_ok(hipMemcpy2D(C->lstate.ptr + LS_HWM * 64, pitch, hwm.data(), row, row, nw,
                                          hipMemcpyHostToDevice), "write marks"))
    return -1;
  return resumed.load() + grown;
}

}  // namespace wbh
