// jit.cpp -- compiled straight-line runs for the V-frame threaded core (jit.h).
//
// Register contract (gen_tc.py): frame cell i = v[128 + i]; PAGES v105, MEM v[106:107],
// HWM v101, v117 = 0; temps v108-v121, v126-v127, s68-s69, s[74:75]; PCOFF s62, OTHER
// s63, CNT s65, the code base s[60:61], bank A s[76:83] / bank B s[84:91], bank-A
// handler base s[70:71] (slot 0 = the xh exit stub, +TC_JIT_XS = xs). Every instruction
// below does what its threaded-core handler does (gen_tc.py specs), with the cell
// numbers and immediates folded in; instruction semantics: dbc_step.inc.
#include "jit.h"

#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <mutex>
#include <tuple>

#include "frontend.h"
#include "tc_slots.h"

namespace wb {

namespace {

constexpr uint32_t kMinRun = 3;   // shorter runs gain less than the entry/exit costs
constexpr uint32_t kMaxRun = 1500;   // keeps a run's branches to its exit stubs in range
constexpr uint32_t kMaxBrTable = 32;   // br_table entries compiled as a compare chain

const char *const PAGES = "v105", *const MEM = "v[106:107]", *const HWM = "v101";
const char *const A0 = "v108", *const A1 = "v109", *const AP = "v[108:109]";
const char *const B0 = "v110", *const B1 = "v111", *const BP = "v[110:111]";
const char *const R0 = "v114", *const R1 = "v115", *const RP = "v[114:115]";
const char *const W0 = "v116", *const WP = "v[116:117]";   // v117 stays 0
const char *const X0 = "v118", *const X1 = "v119", *const XP = "v[118:119]";
const char *const Y0 = "v120", *const Y1 = "v121";
const char *const Z0 = "v126", *const Z1 = "v127", *const ZP = "v[126:127]";
const char *const T2 = "s[74:75]";

uint16_t op_of(const DInstr &I) { return uint16_t(I.w0 & 0x7FFFu); }

bool is_store_op(uint16_t op) {
  return op == OP_ST8 || op == OP_ST16 || op == OP_ST32 || op == OP_ST64 || op == OP_ST128;
}

uint32_t mem_bytes(uint16_t op) {
  switch (op) {
    case OP_LD8S32: case OP_LD8U32: case OP_LD8S64: case OP_LD8U64: case OP_ST8: return 1;
    case OP_LD16S32: case OP_LD16U32: case OP_LD16S64: case OP_LD16U64: case OP_ST16: return 2;
    case OP_LD32: case OP_LD32S64: case OP_LD32U64: case OP_ST32: return 4;
    case OP_LD64: case OP_ST64: return 8;
    case OP_LD128: case OP_ST128: return 16;
    default: return 0;
  }
}

// Memories past the first (MultiMemories; frontend.cpp do_load / do_store): XLD a, k -> c
// and XST a, b -> memory c carry the memory-0 op in D. xmop = that op (0 for anything else).
bool load_wide_op(uint16_t op) {
  return op == OP_LD8S64 || op == OP_LD8U64 || op == OP_LD16S64 || op == OP_LD16U64 ||
         op == OP_LD32S64 || op == OP_LD32U64 || op == OP_LD64;
}
uint16_t xmop(const DInstr &I) {
  const uint16_t op = uint16_t(I.w0 & 0x7FFFu);
  return op == OP_XLD || op == OP_XST ? uint16_t(I.w2 >> 16) : uint16_t(0);
}
// The word offsets of the extra memories in a lane's block (batch_ctx.h xinfo_h: memory k
// at word xinfo[2 (k - 1)]), for the jit_source call that is compiling (null in dry runs)
thread_local const std::vector<uint32_t> *g_xinfo = nullptr;
thread_local uint32_t g_xlog = 0;   // (their granule: 4 << g_xlog bytes, KParams::xlog)
// the first memory's page limit (jit_source's mem_pages): at most kMadPages, a lane's
// granule address fits 32 bits (granule_addr)
thread_local uint32_t g_mem_pages = 65536;
constexpr uint32_t kMadPages = 1000;

// compare ops: VOPC suffix (32-bit form; the 64-bit form appends "64" to the type)
const char *cmp_kind(uint16_t k) {   // k: 0 EQ, 1 NE, 2 LT_S, 3 LT_U, 4 GT_S, 5 GT_U, 6 LE_S, 7 LE_U, 8 GE_S, 9 GE_U
  static const char *const n[] = {"eq_u", "ne_u", "lt_i", "lt_u", "gt_i", "gt_u", "le_i", "le_u", "ge_i", "ge_u"};
  return n[k];
}
uint16_t cmp_swap(uint16_t k) {   // a CMP b == b CMP' a
  static const uint16_t s[] = {0, 1, 4, 5, 2, 3, 8, 9, 6, 7};
  return s[k];
}

struct Em {
  std::string o;
  uint32_t g = 0;        // granule log
  uint32_t run = 0;      // run index (label suffix)
  uint32_t pc = 0;       // instruction being compiled
  uint32_t done = 0;     // wasm instructions retired before it (within the run)
  uint64_t cdone = 0;    // their gas (metered contexts)
  bool metered = false;
  bool pend[256] = {};   // cells with a global load in flight
  bool any = false;
  // Counted waits: vector-memory operations complete in issue order (loads and stores
  // alike: MI355X_MICROARCH.md "vmcnt"), so waiting for the load into cell c leaves the
  // operations issued after it in flight: vmcnt(nvm - 1 - seq[c]). nvm counts the
  // operations this code issued since its last vmcnt(0) (code that issues others waits
  // for them itself, which only makes these counts stricter).
  uint32_t seq[256] = {};
  uint32_t nvm = 0;
  uint32_t basev = 122;   // the current access group's base pair (BASE or v[124:125])
  struct Stub { std::string lab; uint32_t pc, done; uint64_t cdone; };
  std::vector<Stub> stubs;
  const struct MemGroup *group = nullptr;   // set on a group's first access (group_check)
  uint32_t fb = 0;                          // frame base (Program::global_cells)
  const Program *prog = nullptr;

  void l(const char *fmt, ...) __attribute__((format(printf, 2, 3))) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    o += buf;
    o += '\n';
  }
  // Inlined calls (jit_source): the callee's cells from the frame base on live `shift`
  // cells higher, above the caller's live cells (globals stay).
  uint32_t shift = 0;
  uint32_t sc(uint32_t c) const { return (shift && c >= fb) ? c + shift : c; }
  // (one cell may be renamed to another VGPR for one instruction: a forwarded store's
  // value computed straight into its word's VGPR)
  int64_t alias_cell = -1;
  uint32_t alias_reg = 0;
  // (and cells whose value is a forwarded word read straight from its VGPR until they
  // are written: amap cell -> VGPR)
  std::map<uint32_t, uint32_t> amap;
  std::string V(uint32_t c) const {
    if (int64_t(c) == alias_cell) return "v" + std::to_string(alias_reg);
    if (!amap.empty()) {
      auto it = amap.find(c);
      if (it != amap.end()) return "v" + std::to_string(it->second);
    }
    return "v" + std::to_string(128 + sc(c));
  }
  void materialize(uint32_t c) {   // the cell's own register gets its aliased value
    auto it = amap.find(c);
    if (it == amap.end()) return;
    l("v_mov_b32 v%u, v%u", 128 + sc(c), it->second);
    amap.erase(it);
  }
  void before_write(uint32_t reg) {   // VGPR reg changes: cells aliased to it get it first
    std::vector<uint32_t> cells;
    for (const auto &kv : amap)
      if (kv.second == reg) cells.push_back(kv.first);
    for (uint32_t c : cells) materialize(c);
  }
  std::string P(uint32_t c) const {
    return "v[" + std::to_string(128 + sc(c)) + ":" + std::to_string(129 + sc(c)) + "]";
  }
  const char *v(uint32_t c) {   // (short-lived: valid until the next call)
    static thread_local std::string s[8];
    static thread_local int k = 0;
    k = (k + 1) & 7;
    s[k] = V(c);
    return s[k].c_str();
  }
  const char *p(uint32_t c) {
    static thread_local std::string s[8];
    static thread_local int k = 0;
    k = (k + 1) & 7;
    s[k] = P(c);
    return s[k].c_str();
  }
  // wait for loads in flight into any of these cells (read after load, write after load)
  void sync(std::initializer_list<uint32_t> cells) {
    if (!any) return;
    int64_t last = -1;
    for (uint32_t c : cells)
      if (c < 256 && pend[c]) last = std::max<int64_t>(last, seq[c]);
    if (last < 0) return;
    const int64_t younger = int64_t(nvm) - 1 - last;
    if (younger <= 0) { drain(); return; }
    l("s_waitcnt vmcnt(%d)", int(std::min<int64_t>(younger, 63)));
    any = false;
    for (uint32_t c = 0; c < 256; c++) {
      if (pend[c] && seq[c] <= uint64_t(last)) pend[c] = false;
      any = any || pend[c];
    }
  }
  void drain() {
    if (!any) return;
    l("s_waitcnt vmcnt(0)");
    for (bool &b : pend) b = false;
    any = false;
    nvm = 0;
  }
  void loaded(uint32_t c) {   // a global load into cell c was just issued
    pend[c] = any = true;
    seq[c] = nvm++;
  }
  std::string base(int half = -1) const {   // the group's base pair, or one half of it
    if (half < 0) return "v[" + std::to_string(basev) + ":" + std::to_string(basev + 1) + "]";
    return "v" + std::to_string(basev + uint32_t(half));
  }
  // the lanes' gas total (v[96:97]) += c
  void gas_add(uint64_t c) {
    if (!metered || !c) return;
    l("s_mov_b32 s68, 0x%x", uint32_t(c));
    l("s_mov_b32 s69, 0x%x", uint32_t(c >> 32));
    l("v_lshl_add_u64 v[96:97], v[96:97], 0, s[68:69]");
  }
  // a 64-bit operand as an aligned VGPR pair (gfx9 tuples start at even registers)
  const char *src64(uint32_t c, const char *lo, const char *hi, const char *pair) {
    if (!(c & 1)) return p(c);
    l("v_mov_b32 %s, %s", lo, v(c));
    l("v_mov_b32 %s, %s", hi, v(c + 1));
    return pair;
  }
  // cells c, c+1 = R
  void put64(uint32_t c) {
    if (!(c & 1)) {
      l("v_mov_b64 %s, %s", p(c), RP);
    } else {
      l("v_mov_b32 %s, %s", v(c), R0);
      l("v_mov_b32 %s, %s", v(c + 1), R1);
    }
  }
  // cells c..c+3 = the four registers (results computed into temporaries first)
  void put128(uint32_t c, const char *const r[4]) {
    for (int k = 0; k < 4; k++)
      if (r[k] != dst[k]) l("v_mov_b32 %s, %s", v(c + k), r[k]);
  }
  // Result registers of a 4-cell result at c whose sources are the cell ranges in `src`
  // ({first, count}): the cells themselves when no source overlaps them (nothing read
  // after the first write can then see it, and a run that leaves before the instruction
  // re-executes it from intact sources), else the temporaries R0 R1 Z0 Z1 (put128 copies
  // them). pair64: the two 64-bit halves as aligned pairs (c even) for f64 / u64 ops.
  std::string dst[4], dstp[2];
  // lanewise: result word (pair) k depends only on word (pair) k of each source and is
  // written after it is read, so a source that IS the result (c..c+3 exactly) may be
  // overwritten in place
  const char *const *res128(uint32_t c, std::initializer_list<std::pair<uint32_t, uint32_t>> src,
                            bool pair64 = false, bool lanewise = false) {
    static const char *const tmp[4] = {R0, R1, Z0, Z1};
    static thread_local const char *out[4];
    bool direct = !(pair64 && (c & 1));
    for (const auto &r : src)
      if (r.first < c + 4 && c < r.first + r.second && !(lanewise && r.first == c && r.second == 4))
        direct = false;
    for (int k = 0; k < 4; k++) {
      dst[k] = direct ? V(c + k) : "";
      out[k] = direct ? dst[k].c_str() : tmp[k];
    }
    dstp[0] = direct ? P(c) : RP;
    dstp[1] = direct ? P(c + 2) : ZP;
    return out;
  }
  // NaN results fixed in place (an out-of-line block, taken only when some active lane's
  // result is a NaN) to what the reference's x86 build produces: the first NaN operand,
  // quieted, else the default NaN with the sign bit set (dbc_ops.h nan_fix32/64). The
  // sources must be intact (results in temporaries or cells that overlap no source).
  // Items: result register (w 32) or lo/hi registers and the aligned pair (w 64), and the
  // source cells a, b.
  struct NanItem { std::string lo, hi, pair; uint32_t a, b; };
  std::string tail;   // out-of-line code of the run (placed after it)
  int nfix = 0;
  // A run that starts with a POST_CALL (restoring cells) and ends with a RET reads the
  // RET's return record together with the restored cells (one LDS wait instead of two):
  // ret_pf asks POST_CALL to issue it into v113, ret_pf_done tells RET it is there
  bool ret_pf = false, ret_pf_done = false;
  const std::vector<uint8_t> *nanobs = nullptr;   // nan_observable(), per pc
  bool nan_needed() const { return !(nanobs && pc < nanobs->size() && !(*nanobs)[pc]); }
  void nan_fix(const std::vector<NanItem> &items, int w) {
    if (nanobs && pc < nanobs->size() && !(*nanobs)[pc]) return;   // payload never observed
    const std::string id = std::to_string(run) + "_" + std::to_string(nfix++);
    bool first = true;
    for (const auto &it : items) {
      const std::string &r = w == 64 ? it.pair : it.lo;
      l("v_cmp_u_f%d_e64 %s, %s, %s", w, first ? T2 : "vcc", r.c_str(), r.c_str());
      if (!first) l("s_or_b64 %s, %s, vcc", T2, T2);
      first = false;
    }
    l("s_and_b64 %s, %s, exec", T2, T2);
    l("s_cbranch_scc1 Lnf%s", id.c_str());
    l("Lnr%s:", id.c_str());
    std::string o2;
    o.swap(o2);   // (emit the block into `tail`)
    l("Lnf%s:", id.c_str());
    for (const auto &it : items) {
      if (w == 64) {
        l("v_mov_b32 %s, %s", A0, v(it.a));
        l("v_mov_b32 %s, %s", A1, v(it.a + 1));
        l("v_mov_b32 %s, %s", B0, v(it.b));
        l("v_mov_b32 %s, %s", B1, v(it.b + 1));
        l("v_cmp_u_f64_e64 s[68:69], %s, %s", AP, AP);
        l("v_cmp_u_f64_e64 vcc, %s, %s", BP, BP);
        l("v_mov_b32 %s, 0", X0);
        l("v_mov_b32 %s, 0xfff80000", X1);
        l("v_or_b32_e32 %s, 0x80000, %s", Y1, B1);
        l("v_cndmask_b32_e64 %s, %s, %s, vcc", X0, X0, B0);
        l("v_cndmask_b32_e64 %s, %s, %s, vcc", X1, X1, Y1);
        l("v_or_b32_e32 %s, 0x80000, %s", Y1, A1);
        l("v_cndmask_b32_e64 %s, %s, %s, s[68:69]", X0, X0, A0);
        l("v_cndmask_b32_e64 %s, %s, %s, s[68:69]", X1, X1, Y1);
        l("v_cmp_u_f64_e64 vcc, %s, %s", it.pair.c_str(), it.pair.c_str());
        l("v_cndmask_b32_e64 %s, %s, %s, vcc", it.lo.c_str(), it.lo.c_str(), X0);
        l("v_cndmask_b32_e64 %s, %s, %s, vcc", it.hi.c_str(), it.hi.c_str(), X1);
      } else {
        l("v_cmp_u_f32_e64 s[68:69], %s, %s", v(it.a), v(it.a));
        l("v_cmp_u_f32_e64 vcc, %s, %s", v(it.b), v(it.b));
        l("v_mov_b32 %s, 0xffc00000", X0);
        l("v_or_b32_e32 %s, 0x400000, %s", Y1, v(it.b));
        l("v_cndmask_b32_e64 %s, %s, %s, vcc", X0, X0, Y1);
        l("v_or_b32_e32 %s, 0x400000, %s", Y1, v(it.a));
        l("v_cndmask_b32_e64 %s, %s, %s, s[68:69]", X0, X0, Y1);
        l("v_cmp_u_f32_e64 vcc, %s, %s", it.lo.c_str(), it.lo.c_str());
        l("v_cndmask_b32_e64 %s, %s, %s, vcc", it.lo.c_str(), it.lo.c_str(), X0);
      }
    }
    l("s_branch Lnr%s", id.c_str());
    o.swap(o2);
    tail += o2;
  }
  // leave before instruction pc (the C++ step executes it) when any active lane's T2 bit
  // is set
  std::string leave_if_t2() {
    if (trip) return trip_leave();
    const std::string lab = leave_stub();
    l("s_and_b64 %s, %s, exec", T2, T2);
    l("s_cbranch_scc1 %s", lab.c_str());
    return lab;
  }
  // a leave stub before instruction pc without a test here (the caller branches to it)
  std::string leave_stub() {
    const std::string lab = "Lx" + std::to_string(run) + "_" + std::to_string(stubs.size());
    stubs.push_back(Stub{lab, pc, done, cdone});
    return lab;
  }
  // A run that starts with a POST_CALL and ends with a CALL checks the call stack once at
  // its start, for the deeper of the two (jit_source): both instructions skip their own
  bool call_checked = false;
  // cells holding a splat of an f64 inline constant that was never materialized (jit_source
  // fold_consts): the f64x2 ops reading them take the constant itself
  std::map<uint32_t, std::string> kfold;
  bool fuse_any = false;   // V_ANY_TRUE leaves its OR in R0 only (its cell is dead)
  // an f64x2 compare whose mask only an (also fused) any_true reads for the run's branch:
  // the compare leaves the per-lane "any element true" mask in VCC (s[68:69] holds the
  // first element's) and the any_true emits nothing
  bool cmp_any = false;
  const char *kf(uint32_t c) const {
    auto it = kfold.find(c);
    return it == kfold.end() ? nullptr : it->second.c_str();
  }
  // the run's POST_CALL checked the call stack at its start: a RET later in the run pops
  // below that, so it needs no check of its own
  bool stack_ok = false;
  // Trip mode (jit_source): the lanes of T2 leave alone, before instruction pc -- each
  // records it as its pc (VPC v92) with the instructions the run retired before it (VCNT
  // v93), no longer runs in this trip (TPC v98 = -1) and waits outside the trips as an
  // escape (OUTSIDE s[76:77], ESC s[78:79]: the C++ step executes that instruction);
  // the other lanes go on (past the stage's end when none is left). Out of line.
  bool trip = false;
  // (trip stages, memory 0 below kMadPages) a VGPR holding 63 << (2 + g): granule_addr's
  // multiply-add form
  const char *madk = nullptr;
  // Trip-mode load cache (trip_source): loads whose value a scan's exit left in a VGPR --
  // pc -> {the cache's address VGPR, its value VGPR}: the load becomes a move (the lanes
  // running this code matched the address first) -- and the address VGPRs every store
  // invalidates (-1)
  std::map<uint32_t, std::pair<uint32_t, uint32_t>> fwd;
  std::vector<uint32_t> inval;
  std::string stage_end;   // label: the end of the run's current stage (EXEC = its lanes)
  int nleave = 0;
  std::string trip_leave() {
    const std::string id = std::to_string(run) + "_" + std::to_string(nleave++);
    l("s_and_b64 %s, %s, exec", T2, T2);
    l("s_cbranch_scc1 Llv%s", id.c_str());
    l("Llr%s:", id.c_str());
    std::string o2;
    o.swap(o2);
    l("Llv%s:", id.c_str());
    l("s_andn2_b64 exec, exec, %s", T2);
    l("s_or_b64 s[76:77], s[76:77], %s", T2);
    l("s_or_b64 s[78:79], s[78:79], %s", T2);
    l("s_mov_b64 s[68:69], exec");
    l("s_mov_b64 exec, %s", T2);
    l("v_mov_b32 v92, 0x%x", pc);
    if (done) l("v_add_u32_e32 v93, 0x%x, v93", done);
    l("v_mov_b32 v98, -1");
    l("s_mov_b64 exec, s[68:69]");
    l("s_cbranch_execz %s", stage_end.c_str());
    l("s_branch Llr%s", id.c_str());
    o.swap(o2);
    tail += o2;
    return "Llv" + id;
  }
};

// ---------------------------------------------------------------- linear memory
// Accesses are checked in groups: consecutive loads/stores of a run through the same
// address cell a, which nothing in between writes (jit_groups). The group's first
// access checks all of them at once, as the handlers check one (gen_tc.py mem_check):
// the highest last byte a + (offset + n - 1) must not carry and must lie below
// pages * 64 KiB, and each access must be naturally aligned (4 for 8 bytes). If any
// active lane fails, the run leaves before the group (the C++ step and the handlers then
// meet the failing access themselves). Stores raise the write mark (LS_HWM) once, to one
// past the group's highest stored byte. In the word interleave (g = 0) an aligned word
// access is at MEM + ea * 64: the group computes MEM + a * 64 once (BASE) and each access
// adds offset * 64 in its instruction's offset field.
// (BASE = v[122:123]; a load batch's second group uses v[124:125]: Em::basev)

struct MemGroup {
  uint32_t base = 0;                // address cell
  uint32_t maxlast = 0;             // highest offset + n - 1
  uint64_t store_end = 0;           // highest offset + n of a store (0: no store)
  std::vector<std::pair<uint32_t, uint32_t>> aligns;   // distinct (offset & m, m)
  // (trip load cache, LtF) every access of the group is a 32-bit access at an address a
  // scan window already checked for these lanes: no bounds / alignment test
  bool checked = false;
};

// the group's base pair (word interleave): MEM + a * 64
void group_base(Em &e, const MemGroup &G) {
  if (e.g != 0) return;
  const std::string bp = e.base();
  e.l("v_mov_b32 %s, %s", W0, e.v(G.base));
  e.l("v_lshlrev_b64 %s, 6, %s", bp.c_str(), WP);
  e.l("v_lshl_add_u64 %s, %s, 0, %s", bp.c_str(), bp.c_str(), MEM);
}

void group_check(Em &e, const MemGroup &G) {
  const uint32_t a = G.base;
  if (G.checked) {   // (the write mark and the base only)
    if (G.store_end) {
      e.l("s_mov_b32 s69, 0x%x", uint32_t(G.store_end));
      e.l("v_add_u32_e64 %s, %s, s69 clamp", Y1, e.v(a));
      e.l("v_max_u32_e32 %s, %s, %s", HWM, HWM, Y1);
    }
    group_base(e, G);
    return;
  }
  e.l("v_add_co_u32_e32 %s, vcc, 0x%x, %s", X0, G.maxlast, e.v(a));
  e.l("v_lshrrev_b32_e32 %s, 16, %s", X1, X0);
  e.l("v_cmp_ge_u32_e64 %s, %s, %s", T2, X1, PAGES);
  e.l("s_or_b64 %s, %s, vcc", T2, T2);
  for (const auto &am : G.aligns) {
    if (am.first) {
      e.l("v_add_u32_e32 %s, %u, %s", Y0, am.first, e.v(a));
      e.l("v_and_b32_e32 %s, %u, %s", Y0, am.second, Y0);
    } else {
      e.l("v_and_b32_e32 %s, %u, %s", Y0, am.second, e.v(a));
    }
    e.l("v_cmp_ne_u32_e32 vcc, 0, %s", Y0);
    e.l("s_or_b64 %s, %s, vcc", T2, T2);
  }
  e.leave_if_t2();
  if (G.store_end) {   // (cannot carry past 2^32 once the bounds hold; clamp the sum)
    e.l("s_mov_b32 s69, 0x%x", uint32_t(G.store_end));
    e.l("v_add_u32_e64 %s, %s, s69 clamp", Y1, e.v(a));
    e.l("v_max_u32_e32 %s, %s, %s", HWM, HWM, Y1);
  }
  group_base(e, G);
}

// pr = base + the granule address of byte ea: rows of 256 << g bytes, (ea >> (2 + g)) of
// them, + the byte in the granule. With e.madk (the lane's memory below 64 MiB: the offset
// fits 32 bits) that offset is (ea >> s) * (63 << s) + ea, s = 2 + g: one multiply-add and
// one 64-bit add instead of two 64-bit shifts and adds.
void granule_addr(Em &e, const char *pr, const std::string &ea, const char *base) {
  if (e.madk) {
    e.l("v_lshrrev_b32_e32 %s, %u, %s", W0, 2 + e.g, ea.c_str());
    e.l("v_mad_u32_u24 %s, %s, %s, %s", W0, W0, e.madk, ea.c_str());
    e.l("v_lshl_add_u64 %s, %s, 0, %s", pr, WP, base);
    return;
  }
  e.l("v_lshrrev_b32_e32 %s, %u, %s", W0, 2 + e.g, ea.c_str());
  e.l("v_lshlrev_b64 %s, %u, %s", pr, 8 + e.g, WP);
  e.l("v_lshl_add_u64 %s, %s, 0, %s", pr, pr, base);
  e.l("v_bfe_u32 %s, %s, 0, %u", W0, ea.c_str(), 2 + e.g);
  e.l("v_lshl_add_u64 %s, %s, 0, %s", pr, WP, pr);
}

// Address operand(s) of the access at offset imm (n bytes) of the current group: the
// first word's "vaddr, off[ offset:k]" and, for n = 8, the second word's.
void mem_ea(Em &e, uint32_t a, uint32_t imm, uint32_t n, std::string *w1, std::string *w2) {
  if (e.g == 0 && n >= 4) {
    const uint64_t k = uint64_t(imm) * 64u;
    if (k + (n == 8 ? 256 : 0) <= 4095) {
      *w1 = e.base() + ", off offset:" + std::to_string(k);
      *w2 = e.base() + ", off offset:" + std::to_string(k + 256);
    } else {
      e.l("v_add_co_u32_e32 %s, vcc, 0x%x, %s", X0, uint32_t(k), e.base(0).c_str());
      e.l("v_addc_co_u32_e32 %s, vcc, 0x%x, %s, vcc", X1, uint32_t(k >> 32), e.base(1).c_str());
      *w1 = std::string(XP) + ", off";
      *w2 = std::string(XP) + ", off offset:256";
    }
    return;
  }
  // granule rows of 256 << g bytes, (ea >> (2 + g)) of them, + the byte in the granule
  std::string ea = e.V(a);
  if (imm) { e.l("v_add_u32_e32 %s, 0x%x, %s", Y0, imm, e.v(a)); ea = Y0; }
  granule_addr(e, XP, ea, MEM);
  *w1 = std::string(XP) + ", off";
  if (n == 8) {   // ZP = address of the second word (ea + 4: maybe the next granule)
    e.l("v_add_u32_e32 %s, 4, %s", Y1, ea.c_str());
    granule_addr(e, ZP, Y1, MEM);
    *w2 = std::string(ZP) + ", off";
  }
}

// v128 (16 bytes, 4-byte aligned: group_check): the address operand of each of its 4
// words -- in the word interleave offsets from the group's base (or from one computed
// base), else each word's granule address in its own register pair
const char *const WPAIR[4] = {"v[118:119]", "v[126:127]", "v[108:109]", "v[110:111]"};
void mem_ea16(Em &e, uint32_t a, uint32_t imm, std::string w[4]) {
  if (e.g == 0) {
    uint64_t k = uint64_t(imm) * 64u;
    std::string base = e.base();
    if (k + 768 > 4095) {
      e.l("v_add_co_u32_e32 %s, vcc, 0x%x, %s", X0, uint32_t(k), e.base(0).c_str());
      e.l("v_addc_co_u32_e32 %s, vcc, 0x%x, %s, vcc", X1, uint32_t(k >> 32), e.base(1).c_str());
      base = XP;
      k = 0;
    }
    for (int q = 0; q < 4; q++) w[q] = base + ", off offset:" + std::to_string(k + 256u * q);
    return;
  }
  for (int q = 0; q < 4; q++) {
    const std::string pr = WPAIR[q];
    const std::string lo = "v" + pr.substr(2, pr.find(':') - 2);
    e.l("v_add_u32_e32 %s, 0x%x, %s", Y1, imm + 4u * q, e.v(a));
    granule_addr(e, pr.c_str(), Y1, MEM);
    w[q] = pr + ", off";
  }
}

bool emit_load(Em &e, uint16_t op, uint32_t a, uint32_t c, uint32_t imm) {
  const uint32_t n = mem_bytes(op);
  if (n == 16) {   // LD128 (memory.ipp loadValue of a uint128): 4 words into c..c+3
    e.sync({a, c, c + 1, c + 2, c + 3});
    if (e.group) group_check(e, *e.group);
    std::string w[4];
    mem_ea16(e, a, imm, w);
    for (int q = 0; q < 4; q++) {
      e.l("global_load_dword %s, %s", e.v(c + q), w[q].c_str());
      e.loaded(c + q);
    }
    return true;
  }
  if (op == OP_LD32) {
    const auto f = e.fwd.find(e.pc);
    if (f != e.fwd.end()) {   // (trip load cache: these lanes' word is in the value VGPR)
      e.sync({a, c});
      if (e.group) group_check(e, *e.group);
      e.l("v_mov_b32 %s, v%u", e.v(c), f->second.second);
      return true;
    }
  }
  const char *ins = n == 1 ? (op == OP_LD8S32 || op == OP_LD8S64 ? "global_load_sbyte" : "global_load_ubyte")
                    : n == 2 ? (op == OP_LD16S32 || op == OP_LD16S64 ? "global_load_sshort" : "global_load_ushort")
                             : "global_load_dword";
  const bool wide = op == OP_LD8S64 || op == OP_LD8U64 || op == OP_LD16S64 || op == OP_LD16U64 ||
                    op == OP_LD32S64 || op == OP_LD32U64 || op == OP_LD64;
  e.sync({a, c, wide ? c + 1 : c});
  if (e.group) group_check(e, *e.group);
  std::string w1, w2;
  mem_ea(e, a, imm, n, &w1, &w2);
  e.l("%s %s, %s", ins, e.v(c), w1.c_str());
  e.loaded(c);
  if (op == OP_LD64) {
    e.l("global_load_dword %s, %s", e.v(c + 1), w2.c_str());
    e.loaded(c + 1);
  } else if (op == OP_LD8U64 || op == OP_LD16U64 || op == OP_LD32U64) {
    e.l("v_mov_b32 %s, 0", e.v(c + 1));
  } else if (wide) {   // sign extension needs the loaded word
    e.sync({c});
    e.l("v_ashrrev_i32_e32 %s, 31, %s", e.v(c + 1), e.v(c));
  }
  return true;
}

// (data: the register to store from instead of cell b's -- a forwarded word's own VGPR)
bool emit_store(Em &e, uint16_t op, uint32_t a, uint32_t b, uint32_t imm, const char *data = nullptr) {
  const uint32_t n = mem_bytes(op);
  e.drain();   // a store never overtakes a load of this run (same-address ordering)
  if (e.group) group_check(e, *e.group);
  if (n == 16) {   // ST128: 4 words from b..b+3
    std::string w[4];
    mem_ea16(e, a, imm, w);
    for (int q = 0; q < 4; q++) {
      const size_t k = w[q].find(", off");
      e.l("global_store_dword %s, %s%s", w[q].substr(0, k).c_str(), e.v(b + q), w[q].substr(k).c_str());
      e.nvm++;
    }
    for (uint32_t r : e.inval) e.l("v_mov_b32 v%u, -1", r);   // (trip load cache: stale now)
    return true;
  }
  std::string w1, w2;
  mem_ea(e, a, imm, n, &w1, &w2);
  const char *ins = n == 1 ? "global_store_byte" : n == 2 ? "global_store_short" : "global_store_dword";
  const size_t k1 = w1.find(", off"), k2 = w2.find(", off");
  e.l("%s %s, %s%s", ins, w1.substr(0, k1).c_str(), data ? data : e.v(b), w1.substr(k1).c_str());
  e.nvm++;
  if (n == 8) {
    e.l("global_store_dword %s, %s%s", w2.substr(0, k2).c_str(), e.v(b + 1), w2.substr(k2).c_str());
    e.nvm++;
  }
  for (uint32_t r : e.inval) e.l("v_mov_b32 v%u, -1", r);   // (trip load cache: stale now)
  return true;
}

// ---------------------------------------------------------------- extra memories
// XLD / XST on memory k >= 1 (dbc_step.inc OP_XLD / OP_XST; memory.ipp:12-68 on the
// instance getMemInstByIdx names, helper.cpp:206-215). Memory k of every lane lies in
// KParams::xmem as 4-byte words interleaved over the wave's 64 lanes (batch_kernel.hip
// XMEM): the core holds the wave's block in s[98:99], so the lane's word w of memory k is
// at s[98:99] + (xinfo[2 (k - 1)] + w) * 256 + lane * 4 -- the word interleave of memory 0.
// The check is the memory-0 group check on one access with the module's declared minimum
// as the bound: every lane's memory k has at least that many pages (the size starts there
// and only grows), so an access past it -- in bounds on a grown memory or not -- and a
// misaligned one leave before the instruction and the C++ step executes it exactly.
// No write mark: Reset rewrites the extra memories whole.
// RP = the lane's granule 0 of memory k: s[98:99] + xinfo[2 (k - 1)] * 256 + lane * (4 << g)
void xmem_lane_base(Em &e, uint32_t k) {
  const uint64_t woff = g_xinfo && size_t(2 * (k - 1)) < g_xinfo->size() ? (*g_xinfo)[2 * (k - 1)] : 0;
  e.l("v_mbcnt_lo_u32_b32 %s, -1, 0", W0);
  e.l("v_mbcnt_hi_u32_b32 %s, -1, %s", W0, W0);
  e.l("v_lshlrev_b32_e32 %s, %u, %s", W0, 2 + g_xlog, W0);
  if (woff) {
    e.l("s_add_u32 s68, s98, 0x%x", uint32_t(woff << 8));
    e.l("s_addc_u32 s69, s99, 0x%x", uint32_t(woff >> 24));
    e.l("v_lshl_add_u64 %s, %s, 0, s[68:69]", RP, WP);
  } else {
    e.l("v_lshl_add_u64 %s, %s, 0, s[98:99]", RP, WP);
  }
}

bool emit_xmem(Em &e, const DInstr &I) {
  const uint16_t op = op_of(I), mop = xmop(I);
  const bool st = op == OP_XST;
  const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16, c = I.w2 & 0xFFFFu, imm = I.w3;
  const uint32_t k = st ? c : b, n = mem_bytes(mop);
  if (!n || is_store_op(mop) != st || !e.prog || k == 0 || k > e.prog->xmems.size()) return false;
  if (uint64_t(imm) + n - 1 > 0xFFFFFFFFull) return false;
  const uint32_t minp = e.prog->xmems[k - 1].min;
  const bool wide = load_wide_op(mop);
  if (st) e.drain();   // (a store never overtakes a load of this run)
  else e.sync({a, c, wide || n >= 8 ? c + 1 : c, n == 16 ? c + 2 : c, n == 16 ? c + 3 : c});
  // bounds: the last byte a + imm + n - 1 must not carry and must lie below minp pages
  e.l("v_add_co_u32_e32 %s, vcc, 0x%x, %s", X0, imm + n - 1, e.v(a));
  e.l("v_lshrrev_b32_e32 %s, 16, %s", X1, X0);
  e.l("s_mov_b32 s68, 0x%x", minp);
  e.l("v_cmp_le_u32_e64 %s, s68, %s", T2, X1);
  e.l("s_or_b64 %s, %s, vcc", T2, T2);
  const uint32_t m = n >= 4 ? 3 : n - 1;   // (as jit_groups: 4-byte alignment for 8 and 16)
  if (m) {
    if (imm & m) {
      e.l("v_add_u32_e32 %s, %u, %s", Y0, imm & m, e.v(a));
      e.l("v_and_b32_e32 %s, %u, %s", Y0, m, Y0);
    } else {
      e.l("v_and_b32_e32 %s, %u, %s", Y0, m, e.v(a));
    }
    e.l("v_cmp_ne_u32_e32 vcc, 0, %s", Y0);
    e.l("s_or_b64 %s, %s, vcc", T2, T2);
  }
  e.leave_if_t2();
  if (!st && mop == OP_LD32) {
    const auto f = e.fwd.find(e.pc);
    if (f != e.fwd.end()) {   // (trip load cache: these lanes' word is in the value VGPR)
      e.l("v_mov_b32 %s, v%u", e.v(c), f->second.second);
      return true;
    }
  }
  xmem_lane_base(e, k);
  const uint32_t nw = n >= 4 ? n / 4 : 1;   // words (or the one sub-word access)
  std::string adr[4];                       // each one's "vaddr, off[ offset:k]"
  if (g_xlog) {   // granules of 4 << g bytes: each word's granule address in a pair of its own
    static const char *const PR[4] = {"v[118:119]", "v[126:127]", "v[108:109]", "v[110:111]"};
    const uint32_t g = g_xlog;
    for (uint32_t q = 0; q < nw; q++) {
      std::string ea = e.V(a);
      if (imm + 4 * q) { e.l("v_add_u32_e32 %s, 0x%x, %s", Y1, imm + 4 * q, e.v(a)); ea = Y1; }
      e.l("v_lshrrev_b32_e32 %s, %u, %s", W0, 2 + g, ea.c_str());
      e.l("v_lshlrev_b64 %s, %u, %s", PR[q], 8 + g, WP);
      e.l("v_lshl_add_u64 %s, %s, 0, %s", PR[q], PR[q], RP);
      e.l("v_bfe_u32 %s, %s, 0, %u", W0, ea.c_str(), 2 + g);
      e.l("v_lshl_add_u64 %s, %s, 0, %s", PR[q], WP, PR[q]);
      adr[q] = std::string(PR[q]) + ", off";
    }
  } else if (n >= 4) {   // the word interleave: XP = the first word, the others at +256 each
    uint32_t off = 0;
    e.l("v_mov_b32 %s, %s", W0, e.v(a));
    e.l("v_lshlrev_b64 %s, 6, %s", XP, WP);
    e.l("v_lshl_add_u64 %s, %s, 0, %s", XP, XP, RP);
    const uint64_t kk = uint64_t(imm) * 64u;
    if (kk + 256 * (n / 4 - 1) <= 4095) {
      off = uint32_t(kk);
    } else {
      e.l("v_add_co_u32_e32 %s, vcc, 0x%x, %s", X0, uint32_t(kk), X0);
      e.l("v_addc_co_u32_e32 %s, vcc, 0x%x, %s, vcc", X1, uint32_t(kk >> 32), X1);
    }
    for (uint32_t q = 0; q < nw; q++) adr[q] = std::string(XP) + ", off offset:" + std::to_string(off + 256 * q);
  } else {               // the word interleave, a byte or a half: XP = its byte
    std::string ea = e.V(a);
    if (imm) { e.l("v_add_u32_e32 %s, 0x%x, %s", Y0, imm, e.v(a)); ea = Y0; }
    e.l("v_lshrrev_b32_e32 %s, 2, %s", W0, ea.c_str());
    e.l("v_lshlrev_b64 %s, 8, %s", XP, WP);
    e.l("v_lshl_add_u64 %s, %s, 0, %s", XP, XP, RP);
    e.l("v_and_b32_e32 %s, 3, %s", W0, ea.c_str());
    e.l("v_lshl_add_u64 %s, %s, 0, %s", XP, WP, XP);
    adr[0] = std::string(XP) + ", off";
  }
  auto at = [&](uint32_t q) { return adr[q]; };
  if (st) {
    const char *ins = n == 1 ? "global_store_byte" : n == 2 ? "global_store_short" : "global_store_dword";
    for (uint32_t q = 0; q < std::max(1u, n / 4); q++) {
      const std::string ad = at(q);
      const size_t k1 = ad.find(", off");
      e.l("%s %s, %s%s", ins, ad.substr(0, k1).c_str(), e.v(b + q), ad.substr(k1).c_str());
      e.nvm++;
    }
    for (uint32_t r : e.inval) e.l("v_mov_b32 v%u, -1", r);   // (trip load cache: stale now)
    return true;
  }
  const char *ins = n == 1 ? (mop == OP_LD8S32 || mop == OP_LD8S64 ? "global_load_sbyte" : "global_load_ubyte")
                    : n == 2 ? (mop == OP_LD16S32 || mop == OP_LD16S64 ? "global_load_sshort" : "global_load_ushort")
                             : "global_load_dword";
  for (uint32_t q = 0; q < std::max(1u, n / 4); q++) {
    e.l("%s %s, %s", ins, e.v(c + q), at(q).c_str());
    e.loaded(c + q);
  }
  if (mop == OP_LD8U64 || mop == OP_LD16U64 || mop == OP_LD32U64) {
    e.l("v_mov_b32 %s, 0", e.v(c + 1));
  } else if (wide && mop != OP_LD64) {   // sign extension needs the loaded word
    e.sync({c});
    e.l("v_ashrrev_i32_e32 %s, 31, %s", e.v(c + 1), e.v(c));
  }
  return true;
}

// ---------------------------------------------------------------- one instruction
// Returns false when the instruction has no compiled form (the run ends before it).
bool emit(Em &e, const DInstr &I) {
  const uint16_t op = op_of(I);
  const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16, c = I.w2 & 0xFFFFu, d = I.w2 >> 16, imm = I.w3;
  // i32 binary ops: (register form, immediate form); SUB_I as a - imm
  struct Bin { uint16_t rr, ri; const char *ins; int form; };   // form 0 VOP2, 1 shift, 2 VOP3
  static const Bin bins[] = {
      {OP_I32_ADD, OP_I32_ADD_I, "v_add_u32_e32", 0}, {OP_I32_SUB, OP_I32_SUB_I, "v_sub_u32_e32", 0},
      {OP_I32_MUL, OP_I32_MUL_I, "v_mul_lo_u32", 2}, {OP_I32_AND, OP_I32_AND_I, "v_and_b32_e32", 0},
      {OP_I32_OR, OP_I32_OR_I, "v_or_b32_e32", 0}, {OP_I32_XOR, OP_I32_XOR_I, "v_xor_b32_e32", 0},
      {OP_I32_SHL, OP_I32_SHL_I, "v_lshlrev_b32_e32", 1}, {OP_I32_SHR_S, OP_I32_SHR_S_I, "v_ashrrev_i32_e32", 1},
      {OP_I32_SHR_U, OP_I32_SHR_U_I, "v_lshrrev_b32_e32", 1}};
  for (const Bin &x : bins) {
    if (op == x.rr) {
      e.sync({a, b, c});
      if (x.form == 1) e.l("%s %s, %s, %s", x.ins, e.v(c), e.v(b), e.v(a));
      else e.l("%s %s, %s, %s", x.ins, e.v(c), e.v(a), e.v(b));
      return true;
    }
    if (op == x.ri) {
      e.sync({a, c});
      if (x.form == 1) {
        e.l("%s %s, %u, %s", x.ins, e.v(c), imm & 31u, e.v(a));
      } else if (x.form == 2) {
        e.l("s_mov_b32 s68, 0x%x", imm);
        e.l("%s %s, %s, s68", x.ins, e.v(c), e.v(a));
      } else if (op == OP_I32_SUB_I) {
        e.l("v_subrev_u32_e32 %s, 0x%x, %s", e.v(c), imm, e.v(a));
      } else {
        e.l("%s %s, 0x%x, %s", x.ins, e.v(c), imm, e.v(a));
      }
      return true;
    }
  }
  // compares: I32_EQ..I32_GE_U, *_I; I64 likewise
  if ((op >= OP_I32_EQ && op <= OP_I32_GE_U) || (op >= OP_I32_EQ_I && op <= OP_I32_GE_U_I)) {
    const bool ri = op >= OP_I32_EQ_I;
    const uint16_t k = uint16_t(op - (ri ? OP_I32_EQ_I : OP_I32_EQ));
    if (ri) {
      e.sync({a, c});
      e.l("v_cmp_%s32_e32 vcc, 0x%x, %s", cmp_kind(cmp_swap(k)), imm, e.v(a));
    } else {
      e.sync({a, b, c});
      e.l("v_cmp_%s32_e32 vcc, %s, %s", cmp_kind(k), e.v(a), e.v(b));
    }
    e.l("v_cndmask_b32_e64 %s, 0, 1, vcc", e.v(c));
    return true;
  }
  if ((op >= OP_I64_EQ && op <= OP_I64_GE_U) || (op >= OP_I64_EQ_I && op <= OP_I64_GE_U_I)) {
    const bool ri = op >= OP_I64_EQ_I;
    const uint16_t k = uint16_t(op - (ri ? OP_I64_EQ_I : OP_I64_EQ));
    e.sync({a, a + 1, b, b + 1, c});
    const char *x = e.src64(a, A0, A1, AP);
    const char *y;
    std::string kimm;
    if (ri && int32_t(imm) >= -16 && int32_t(imm) <= 64) {   // (an inline constant: sign-extended)
      kimm = std::to_string(int32_t(imm));
      y = kimm.c_str();
    } else if (ri) {
      e.l("v_mov_b32 %s, 0x%x", Z0, imm);
      e.l("v_ashrrev_i32_e32 %s, 31, %s", Z1, Z0);
      y = ZP;
    } else {
      y = e.src64(b, B0, B1, BP);
    }
    e.l("v_cmp_%s64_e64 vcc, %s, %s", cmp_kind(k), x, y);
    e.l("v_cndmask_b32_e64 %s, 0, 1, vcc", e.v(c));
    return true;
  }
  switch (op) {
    case OP_NOP_CNT:
      return true;
    // ---- floating point (results exact IEEE; a NaN result leaves to the C++ step)
    case OP_F32_ADD: case OP_F32_SUB: case OP_F32_MUL: {
      e.sync({a, b, c});
      const char *ins = op == OP_F32_MUL ? "v_mul_f32_e32" : op == OP_F32_SUB ? "v_sub_f32_e32" : "v_add_f32_e32";
      e.l("%s %s, %s, %s", ins, R0, e.v(a), e.v(b));
      e.nan_fix({{R0, "", "", a, b}}, 32);
      e.l("v_mov_b32 %s, %s", e.v(c), R0);
      return true;
    }
    case OP_F64_ADD: case OP_F64_SUB: case OP_F64_MUL: {
      e.sync({a, a + 1, b, b + 1, c, c + 1});
      const char *x = e.src64(a, A0, A1, AP), *y = e.src64(b, B0, B1, BP);
      if (op == OP_F64_MUL) e.l("v_mul_f64 %s, %s, %s", RP, x, y);
      else e.l("v_add_f64 %s, %s, %s%s", RP, x, op == OP_F64_SUB ? "-" : "", y);
      e.nan_fix({{R0, R1, RP, a, b}}, 64);
      e.put64(c);
      return true;
    }
    case OP_F32_EQ: case OP_F32_NE: case OP_F32_LT: case OP_F32_GT: case OP_F32_LE: case OP_F32_GE: {
      static const char *const k[] = {"eq", "neq", "lt", "gt", "le", "ge"};
      e.sync({a, b, c});
      e.l("v_cmp_%s_f32_e32 vcc, %s, %s", k[op - OP_F32_EQ], e.v(a), e.v(b));
      e.l("v_cndmask_b32_e64 %s, 0, 1, vcc", e.v(c));
      return true;
    }
    case OP_F64_EQ: case OP_F64_NE: case OP_F64_LT: case OP_F64_GT: case OP_F64_LE: case OP_F64_GE: {
      static const char *const k[] = {"eq", "neq", "lt", "gt", "le", "ge"};
      e.sync({a, a + 1, b, b + 1, c});
      const char *x = e.src64(a, A0, A1, AP), *y = e.src64(b, B0, B1, BP);
      e.l("v_cmp_%s_f64_e64 vcc, %s, %s", k[op - OP_F64_EQ], x, y);
      e.l("v_cndmask_b32_e64 %s, 0, 1, vcc", e.v(c));
      return true;
    }
    case OP_F32_ABS: case OP_F32_NEG:
      e.sync({a, c});
      e.l("%s %s, 0x%x, %s", op == OP_F32_ABS ? "v_and_b32_e32" : "v_xor_b32_e32", e.v(c),
          op == OP_F32_ABS ? 0x7FFFFFFFu : 0x80000000u, e.v(a));
      return true;
    case OP_F64_ABS: case OP_F64_NEG:
      e.sync({a, a + 1, c, c + 1});
      e.l("%s %s, 0x%x, %s", op == OP_F64_ABS ? "v_and_b32_e32" : "v_xor_b32_e32", R1,
          op == OP_F64_ABS ? 0x7FFFFFFFu : 0x80000000u, e.v(a + 1));
      e.l("v_mov_b32 %s, %s", R0, e.v(a));
      e.put64(c);
      return true;
    case OP_F32_COPYSIGN:
      e.sync({a, b, c});
      e.l("s_mov_b32 s68, 0x7fffffff");
      e.l("v_bfi_b32 %s, s68, %s, %s", e.v(c), e.v(a), e.v(b));
      return true;
    case OP_F64_COPYSIGN:
      e.sync({a, a + 1, b, b + 1, c, c + 1});
      e.l("s_mov_b32 s68, 0x7fffffff");
      e.l("v_bfi_b32 %s, s68, %s, %s", R1, e.v(a + 1), e.v(b + 1));
      e.l("v_mov_b32 %s, %s", R0, e.v(a));
      e.put64(c);
      return true;
    case OP_F64_CONVERT_I32_S: case OP_F64_CONVERT_I32_U:
      e.sync({a, c, c + 1});
      e.l("%s %s, %s", op == OP_F64_CONVERT_I32_S ? "v_cvt_f64_i32_e32" : "v_cvt_f64_u32_e32", RP, e.v(a));
      e.put64(c);
      return true;
    case OP_F32_CONVERT_I32_S: case OP_F32_CONVERT_I32_U:
      e.sync({a, c});
      e.l("%s %s, %s", op == OP_F32_CONVERT_I32_S ? "v_cvt_f32_i32_e32" : "v_cvt_f32_u32_e32", e.v(c), e.v(a));
      return true;
    // ---- SIMD128 (4 cells; results through temporaries R0 R1 Z0 Z1)
    case OP_MOV128: case OP_CONST128: case OP_V_I32X4_SPLAT: case OP_V_F32X4_SPLAT:
    case OP_V_I64X2_SPLAT: case OP_V_F64X2_SPLAT: {
      if (op == OP_CONST128) {
        if (!e.prog || uint64_t(imm) * 4 + 4 > e.prog->vconst.size()) return false;
        e.sync({c, c + 1, c + 2, c + 3});
        for (int k = 0; k < 4; k++) e.l("v_mov_b32 %s, 0x%x", e.v(c + k), e.prog->vconst[imm * 4 + k]);
        return true;
      }
      e.sync({a, a + 1, a + 2, a + 3, c, c + 1, c + 2, c + 3});
      if (op == OP_MOV128 && a == c) return true;
      if (op != OP_MOV128 && a == c) {   // a splat in place: copy the lane into the rest
        const uint32_t w = (op == OP_V_I32X4_SPLAT || op == OP_V_F32X4_SPLAT) ? 1 : 2;
        for (uint32_t k = w; k < 4; k++) e.l("v_mov_b32 %s, %s", e.v(c + k), e.v(a + (k % w)));
        return true;
      }
      const uint32_t na = op == OP_MOV128 ? 4 : (op == OP_V_I32X4_SPLAT || op == OP_V_F32X4_SPLAT) ? 1 : 2;
      const char *const *rr = e.res128(c, {{a, na}});
      for (int k = 0; k < 4; k++) {
        const uint32_t src = op == OP_MOV128 ? a + k
                             : (op == OP_V_I32X4_SPLAT || op == OP_V_F32X4_SPLAT) ? a : a + (k & 1);
        e.l("v_mov_b32 %s, %s", rr[k], e.v(src));
      }
      e.put128(c, rr);
      return true;
    }
    case OP_V_AND: case OP_V_OR: case OP_V_XOR: case OP_V_I32X4_ADD: case OP_V_I32X4_SUB:
    case OP_V_I32X4_MUL: {
      const char *ins = op == OP_V_AND ? "v_and_b32_e32" : op == OP_V_OR ? "v_or_b32_e32"
                        : op == OP_V_XOR ? "v_xor_b32_e32" : op == OP_V_I32X4_ADD ? "v_add_u32_e32"
                        : op == OP_V_I32X4_SUB ? "v_sub_u32_e32" : "v_mul_lo_u32";
      e.sync({a, a + 1, a + 2, a + 3, b, b + 1, b + 2, b + 3, c, c + 1, c + 2, c + 3});
      const char *const *r = e.res128(c, {{a, 4}, {b, 4}}, false, true);
      for (int k = 0; k < 4; k++) e.l("%s %s, %s, %s", ins, r[k], e.v(a + k), e.v(b + k));
      e.put128(c, r);
      return true;
    }
    case OP_V_I64X2_ADD: case OP_V_I64X2_SUB: case OP_V_I64X2_EQ: {
      e.sync({a, a + 1, a + 2, a + 3, b, b + 1, b + 2, b + 3, c, c + 1, c + 2, c + 3});
      const char *const *r = e.res128(c, {{a, 4}, {b, 4}}, false, true);
      for (int k = 0; k < 2; k++) {
        const uint32_t x = a + 2 * k, y = b + 2 * k;
        if (op == OP_V_I64X2_SUB) {
          e.l("v_sub_co_u32_e32 %s, vcc, %s, %s", r[2 * k], e.v(x), e.v(y));
          e.l("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc", r[2 * k + 1], e.v(x + 1), e.v(y + 1));
        } else if (op == OP_V_I64X2_ADD) {
          e.l("v_add_co_u32_e32 %s, vcc, %s, %s", r[2 * k], e.v(x), e.v(y));
          e.l("v_addc_co_u32_e32 %s, vcc, %s, %s, vcc", r[2 * k + 1], e.v(x + 1), e.v(y + 1));
        } else {
          const char *xx = e.src64(x, A0, A1, AP), *yy = e.src64(y, B0, B1, BP);
          e.l("v_cmp_eq_u64_e64 vcc, %s, %s", xx, yy);
          e.l("v_cndmask_b32_e64 %s, 0, -1, vcc", r[2 * k]);
          e.l("v_mov_b32 %s, %s", r[2 * k + 1], r[2 * k]);
        }
      }
      e.put128(c, r);
      return true;
    }
    case OP_V_F32X4_ADD: case OP_V_F32X4_SUB: case OP_V_F32X4_MUL: {
      const char *ins = op == OP_V_F32X4_MUL ? "v_mul_f32_e32" : op == OP_V_F32X4_SUB ? "v_sub_f32_e32" : "v_add_f32_e32";
      e.sync({a, a + 1, a + 2, a + 3, b, b + 1, b + 2, b + 3, c, c + 1, c + 2, c + 3});
      const char *const *r = e.res128(c, {{a, 4}, {b, 4}}, false, !e.nan_needed());
      for (int k = 0; k < 4; k++) e.l("%s %s, %s, %s", ins, r[k], e.v(a + k), e.v(b + k));
      e.nan_fix({{r[0], "", "", a, b}, {r[1], "", "", a + 1, b + 1}, {r[2], "", "", a + 2, b + 2},
                 {r[3], "", "", a + 3, b + 3}}, 32);
      e.put128(c, r);
      return true;
    }
    case OP_V_F64X2_ADD: case OP_V_F64X2_SUB: case OP_V_F64X2_MUL: {
      e.sync({a, a + 1, a + 2, a + 3, b, b + 1, b + 2, b + 3, c, c + 1, c + 2, c + 3});
      const char *const *r = e.res128(c, {{a, 4}, {b, 4}}, true, !e.nan_needed());
      const std::string res[2] = {e.dstp[0], e.dstp[1]};
      for (int k = 0; k < 2; k++) {
        const char *x = e.kf(a + 2 * k) ? e.kf(a + 2 * k) : e.src64(a + 2 * k, A0, A1, AP);
        const char *y = e.kf(b + 2 * k) ? e.kf(b + 2 * k) : e.src64(b + 2 * k, B0, B1, BP);
        if (op == OP_V_F64X2_MUL) e.l("v_mul_f64 %s, %s, %s", res[k].c_str(), x, y);
        else if (op == OP_V_F64X2_SUB && e.kf(b + 2 * k))   // (a folded constant: negate it)
          e.l("v_add_f64 %s, %s, %s", res[k].c_str(), x, y[0] == '-' ? y + 1 : ("-" + std::string(y)).c_str());
        else e.l("v_add_f64 %s, %s, %s%s", res[k].c_str(), x, op == OP_V_F64X2_SUB ? "-" : "", y);
      }
      e.nan_fix({{r[0], r[1], res[0], a, b}, {r[2], r[3], res[1], a + 2, b + 2}}, 64);
      e.put128(c, r);
      return true;
    }
    case OP_V_F32X4_EQ: case OP_V_F32X4_NE: case OP_V_F32X4_LT: case OP_V_F32X4_GT:
    case OP_V_F32X4_LE: case OP_V_F32X4_GE: {
      static const char *const k[] = {"eq", "neq", "lt", "gt", "le", "ge"};
      e.sync({a, a + 1, a + 2, a + 3, b, b + 1, b + 2, b + 3, c, c + 1, c + 2, c + 3});
      const char *const *r = e.res128(c, {{a, 4}, {b, 4}}, false, true);
      for (int q = 0; q < 4; q++) {
        e.l("v_cmp_%s_f32_e32 vcc, %s, %s", k[op - OP_V_F32X4_EQ], e.v(a + q), e.v(b + q));
        e.l("v_cndmask_b32_e64 %s, 0, -1, vcc", r[q]);
      }
      e.put128(c, r);
      return true;
    }
    case OP_V_F64X2_EQ: case OP_V_F64X2_NE: case OP_V_F64X2_LT: case OP_V_F64X2_GT:
    case OP_V_F64X2_LE: case OP_V_F64X2_GE: {
      static const char *const k[] = {"eq", "neq", "lt", "gt", "le", "ge"};
      e.sync({a, a + 1, a + 2, a + 3, b, b + 1, b + 2, b + 3, c, c + 1, c + 2, c + 3});
      const char *const *r = e.res128(c, {{a, 4}, {b, 4}}, false, true);
      for (int q = 0; q < 2; q++) {
        const char *x = e.kf(a + 2 * q) ? e.kf(a + 2 * q) : e.src64(a + 2 * q, A0, A1, AP);
        const char *y = e.kf(b + 2 * q) ? e.kf(b + 2 * q) : e.src64(b + 2 * q, B0, B1, BP);
        const char *m = e.cmp_any && q == 0 ? "s[68:69]" : "vcc";
        e.l("v_cmp_%s_f64_e64 %s, %s, %s", k[op - OP_V_F64X2_EQ], m, x, y);
        e.l("v_cndmask_b32_e64 %s, 0, -1, %s", r[2 * q], m);
        e.l("v_mov_b32 %s, %s", r[2 * q + 1], r[2 * q]);
      }
      e.put128(c, r);
      if (e.cmp_any) e.l("s_or_b64 vcc, vcc, s[68:69]");   // lanes with any element true
      return true;
    }
    case OP_V_BITSELECT: {   // (a & d) | (b & ~d) per bit: v_bfi_b32(d, a, b)
      e.sync({a, a + 1, a + 2, a + 3, b, b + 1, b + 2, b + 3, d, d + 1, d + 2, d + 3, c, c + 1, c + 2, c + 3});
      const char *const *r = e.res128(c, {{a, 4}, {b, 4}, {d, 4}}, false, true);
      for (int k = 0; k < 4; k++) e.l("v_bfi_b32 %s, %s, %s, %s", r[k], e.v(d + k), e.v(a + k), e.v(b + k));
      e.put128(c, r);
      return true;
    }
    case OP_V_I32X4_SHL: case OP_V_I32X4_SHR_S: case OP_V_I32X4_SHR_U: {   // count mod 32
      e.sync({a, a + 1, a + 2, a + 3, b, c, c + 1, c + 2, c + 3});
      const char *ins = op == OP_V_I32X4_SHL ? "v_lshlrev_b32_e32" : op == OP_V_I32X4_SHR_U ? "v_lshrrev_b32_e32"
                                                                                         : "v_ashrrev_i32_e32";
      e.l("v_and_b32_e32 %s, 31, %s", Y0, e.v(b));
      const char *const *r = e.res128(c, {{a, 4}}, false, true);
      for (int k = 0; k < 4; k++) e.l("%s %s, %s, %s", ins, r[k], Y0, e.v(a + k));
      e.put128(c, r);
      return true;
    }
    case OP_V_I64X2_SHL: case OP_V_I64X2_SHR_S: case OP_V_I64X2_SHR_U: {   // count mod 64
      e.sync({a, a + 1, a + 2, a + 3, b, c, c + 1, c + 2, c + 3});
      const char *ins = op == OP_V_I64X2_SHL ? "v_lshlrev_b64" : op == OP_V_I64X2_SHR_U ? "v_lshrrev_b64"
                                                                                     : "v_ashrrev_i64";
      e.l("v_and_b32_e32 %s, 63, %s", Y0, e.v(b));
      const char *const *r = e.res128(c, {{a, 4}}, true, true);
      (void)r;
      const std::string res[2] = {e.dstp[0], e.dstp[1]};
      for (int k = 0; k < 2; k++) {
        const char *x = e.src64(a + 2 * k, A0, A1, AP);
        e.l("%s %s, %s, %s", ins, res[k].c_str(), Y0, x);
      }
      e.put128(c, r);
      return true;
    }
    case OP_V_ANY_TRUE:
      if (e.cmp_any) return true;   // (the compare before it left the lane mask in VCC)
      e.sync({a, a + 1, a + 2, a + 3, c});
      e.l("v_or3_b32 %s, %s, %s, %s", R0, e.v(a), e.v(a + 1), e.v(a + 2));
      e.l("v_or_b32_e32 %s, %s, %s", R0, R0, e.v(a + 3));
      if (e.fuse_any) return true;   // (jit_source: the branch after it tests R0 itself)
      e.l("v_cmp_ne_u32_e32 vcc, 0, %s", R0);
      e.l("v_cndmask_b32_e64 %s, 0, 1, vcc", e.v(c));
      return true;
    case OP_V_I32X4_BITMASK:
      e.sync({a, a + 1, a + 2, a + 3, c});
      e.l("v_lshrrev_b32_e32 %s, 31, %s", R0, e.v(a));
      for (uint32_t q = 1; q < 4; q++) {
        e.l("v_lshrrev_b32_e32 %s, 31, %s", R1, e.v(a + q));
        e.l("v_lshl_or_b32 %s, %s, %u, %s", R0, R1, q, R0);
      }
      e.l("v_mov_b32 %s, %s", e.v(c), R0);
      return true;
    case OP_V_EXTRACT32:
      e.sync({a + d, c});
      if (a + d != c) e.l("v_mov_b32 %s, %s", e.v(c), e.v(a + d));
      return true;
    case OP_V_EXTRACT64:
      e.sync({a + 2 * d, a + 2 * d + 1, c, c + 1});
      e.l("v_mov_b32 %s, %s", R0, e.v(a + 2 * d));
      e.l("v_mov_b32 %s, %s", R1, e.v(a + 2 * d + 1));
      e.put64(c);
      return true;
    case OP_V_REPLACE64: {
      if (d > 1) return false;
      e.sync({a, a + 1, a + 2, a + 3, b, b + 1, c, c + 1, c + 2, c + 3});
      const char *const *r = e.res128(c, {{a, 4}, {b, 2}});
      for (uint32_t q = 0; q < 4; q++)
        e.l("v_mov_b32 %s, %s", r[q], e.v(q / 2 == d ? b + (q & 1) : a + q));
      e.put128(c, r);
      return true;
    }
    case OP_POST_CALL: {   // gen_tc.py post_call_body_v: results fb.. -> L.., restore [fb, L)
      const uint32_t L = a, r = b, fb = e.fb;
      if (L < e.fb || uint64_t(L) + r > TC_VF_CELLS) return false;
      e.drain();
      if (!e.call_checked) {
        e.l("v_cmp_lt_u32_e64 %s, s93, v102", T2);   // call stack slots past LDS: the C++ step
        e.leave_if_t2();
      }
      e.stack_ok = !e.trip;
      for (uint32_t k = r; k-- > 0;)
        if (L != fb) e.l("v_mov_b32 %s, %s", e.v(L + k), e.v(fb + k));
      if (L > fb) {
        e.l("v_subrev_u32_e32 v102, %u, v102", L - fb);
        e.l("v_lshl_add_u32 %s, v102, 8, v103", X0);
        for (uint32_t k = 0; k < L - fb; k++) e.l("ds_read_b32 %s, %s offset:%u", e.v(fb + k), X0, k * 256u);
        if (e.ret_pf) {   // the run's RET record, one slot below the restored cells
          e.l("v_subrev_u32_e32 %s, 0x100, %s", X1, X0);
          e.l("ds_read_b32 v113, %s", X1);
          e.ret_pf_done = true;
        }
        e.l("s_waitcnt lgkmcnt(0)");
      }
      return true;
    }
    case OP_TAIL_CALL:   // the last instruction of a run (emit_tail_call)
    case OP_CALL: {   // the last instruction of a run (emit_call)
      const uint32_t L = a, nargs = b, nloc = c, fb = e.fb;
      return L >= fb && L < TC_VF_CELLS && imm < (1u << 26) && uint64_t(L) + nargs <= TC_VF_CELLS &&
             uint64_t(fb) + nargs + nloc <= TC_VF_CELLS && L - fb < 255;
    }
    case OP_JMP: case OP_BR_IF: case OP_BR_UNLESS:
    case OP_BR_EQ: case OP_BR_NE: case OP_BR_LT_S: case OP_BR_LT_U: case OP_BR_GT_S: case OP_BR_GT_U:
    case OP_BR_LE_S: case OP_BR_LE_U: case OP_BR_GE_S: case OP_BR_GE_U:
    case OP_BR_EQ_I: case OP_BR_NE_I: case OP_BR_LT_S_I: case OP_BR_LT_U_I: case OP_BR_GT_S_I:
    case OP_BR_GT_U_I: case OP_BR_LE_S_I: case OP_BR_LE_U_I: case OP_BR_GE_S_I: case OP_BR_GE_U_I:
      // the last instruction of a run (emit_branch); as tc.cpp: a taken count >= 0
      return int32_t((I.w0 >> 16) & 0xFFu) + int32_t(int16_t(d)) >= 0 && imm < (1u << 26);
    case OP_BR_TABLE: {   // the last instruction of a run (emit_br_table): small tables
      if (!e.prog || b >= kMaxBrTable || (uint64_t(imm) + b + 1) * 2 > e.prog->brtab.size()) return false;
      for (uint32_t k = 0; k <= b; k++) {
        const uint32_t t = e.prog->brtab[2 * (imm + k)];
        const int32_t tc = int32_t(e.prog->brtab[2 * (imm + k) + 1]);
        if (t >= (1u << 26) || int32_t((I.w0 >> 16) & 0xFFu) + tc < 0) return false;
      }
      return true;
    }
    case OP_RET:    // the last instruction of a run (emit_ret)
      return e.fb < TC_VF_CELLS && uint64_t(a) + b <= TC_VF_CELLS;
    case OP_ZERO_LOCALS:   // a = first cell, b = count
      if (uint64_t(a) + b > TC_VF_CELLS) return false;
      for (uint32_t k = 0; k < b; k++) {
        e.sync({a + k});
        e.l("v_mov_b32 %s, 0", e.v(a + k));
      }
      return true;
    case OP_MOV32:
      e.sync({a, c});
      if (a != c) e.l("v_mov_b32 %s, %s", e.v(c), e.v(a));
      return true;
    case OP_MOV64:
      e.sync({a, a + 1, c, c + 1});
      if (a == c) return true;
      if (!(a & 1) && !(c & 1)) {
        e.l("v_mov_b64 %s, %s", e.p(c), e.p(a));
      } else if (c > a) {   // overlapping copies: the word that would be overwritten first
        e.l("v_mov_b32 %s, %s", e.v(c + 1), e.v(a + 1));
        e.l("v_mov_b32 %s, %s", e.v(c), e.v(a));
      } else {
        e.l("v_mov_b32 %s, %s", e.v(c), e.v(a));
        e.l("v_mov_b32 %s, %s", e.v(c + 1), e.v(a + 1));
      }
      return true;
    case OP_CONST32:
      e.sync({c});
      e.l("v_mov_b32 %s, 0x%x", e.v(c), imm);
      return true;
    case OP_CONST64:
      e.sync({c, c + 1});
      e.l("v_mov_b32 %s, 0x%x", e.v(c), imm);
      e.l("v_mov_b32 %s, 0x%x", e.v(c + 1), I.w1);
      return true;
    case OP_SELECT32:
      e.sync({a, b, c, d});
      e.l("v_cmp_ne_u32_e32 vcc, 0, %s", e.v(d));
      e.l("v_cndmask_b32_e32 %s, %s, %s, vcc", e.v(c), e.v(b), e.v(a));
      return true;
    case OP_SELECT64:
      e.sync({a, a + 1, b, b + 1, c, c + 1, d});
      e.l("v_cmp_ne_u32_e32 vcc, 0, %s", e.v(d));
      e.l("v_cndmask_b32_e32 %s, %s, %s, vcc", R0, e.v(b), e.v(a));
      e.l("v_cndmask_b32_e32 %s, %s, %s, vcc", R1, e.v(b + 1), e.v(a + 1));
      e.put64(c);
      return true;
    case OP_I32_ROTR:
      e.sync({a, b, c});
      e.l("v_alignbit_b32 %s, %s, %s, %s", e.v(c), e.v(a), e.v(a), e.v(b));
      return true;
    case OP_I32_ROTL:
      e.sync({a, b, c});
      e.l("v_sub_u32_e32 %s, 0, %s", X0, e.v(b));
      e.l("v_alignbit_b32 %s, %s, %s, %s", e.v(c), e.v(a), e.v(a), X0);
      return true;
    case OP_I32_ROTR_I: case OP_I32_ROTL_I: {
      e.sync({a, c});
      const uint32_t k = op == OP_I32_ROTR_I ? imm & 31u : (32u - (imm & 31u)) & 31u;
      e.l("v_alignbit_b32 %s, %s, %s, %u", e.v(c), e.v(a), e.v(a), k);
      return true;
    }
    case OP_I32_EQZ:
      e.sync({a, c});
      e.l("v_cmp_eq_u32_e32 vcc, 0, %s", e.v(a));
      e.l("v_cndmask_b32_e64 %s, 0, 1, vcc", e.v(c));
      return true;
    case OP_I32_CLZ: case OP_I32_CTZ:
      e.sync({a, c});
      e.l("%s %s, %s", op == OP_I32_CLZ ? "v_ffbh_u32_e32" : "v_ffbl_b32_e32", X0, e.v(a));
      e.l("v_min_u32_e32 %s, 32, %s", e.v(c), X0);
      return true;
    case OP_I32_POPCNT:
      e.sync({a, c});
      e.l("v_bcnt_u32_b32 %s, %s, 0", e.v(c), e.v(a));
      return true;
    case OP_I32_EXT8S: case OP_I32_EXT16S:
      e.sync({a, c});
      e.l("v_bfe_i32 %s, %s, 0, %u", e.v(c), e.v(a), op == OP_I32_EXT8S ? 8u : 16u);
      return true;
    case OP_I32_ADD3:
      e.sync({a, b, c, d});
      e.l("v_add3_u32 %s, %s, %s, %s", e.v(c), e.v(a), e.v(b), e.v(d));
      return true;
    case OP_I32_XOR_ROTR_I: case OP_I32_XOR_ROTL_I: {
      e.sync({a, b, c});
      const uint32_t k = op == OP_I32_XOR_ROTR_I ? imm & 31u : (32u - (imm & 31u)) & 31u;
      e.l("v_xor_b32_e32 %s, %s, %s", e.v(c), e.v(a), e.v(b));
      e.l("v_alignbit_b32 %s, %s, %s, %u", e.v(c), e.v(c), e.v(c), k);
      return true;
    }
    case OP_I32_ADD_XROTR_I: case OP_I32_ADD3_XROTR_I: {
      // s = a + b (+ d); c = s; y = rotr(y ^ s, k) with y read before c is written
      const bool three = op == OP_I32_ADD3_XROTR_I;
      const uint32_t y = three ? imm & 0xFFFFu : d, k = (three ? imm >> 16 : imm) & 31u;
      e.sync({a, b, c, d, y});
      const std::string s = c == y ? std::string(R0) : e.V(c);
      if (three) e.l("v_add3_u32 %s, %s, %s, %s", s.c_str(), e.v(a), e.v(b), e.v(d));
      else e.l("v_add_u32_e32 %s, %s, %s", s.c_str(), e.v(a), e.v(b));
      // (no temporaries when c != y: the scheduler below then sees only frame cells)
      e.l("v_xor_b32_e32 %s, %s, %s", e.v(y), e.v(y), s.c_str());
      e.l("v_alignbit_b32 %s, %s, %s, %u", e.v(y), e.v(y), e.v(y), k);
      return true;
    }
    // ---- i64 (b operand of *_I: imm sign-extended)
    case OP_I64_ADD: case OP_I64_ADD_I: case OP_I64_SUB: case OP_I64_SUB_I:
    case OP_I64_MUL: case OP_I64_MUL_I: case OP_I64_AND: case OP_I64_AND_I:
    case OP_I64_OR: case OP_I64_OR_I: case OP_I64_XOR: case OP_I64_XOR_I: {
      const bool ri = op == OP_I64_ADD_I || op == OP_I64_SUB_I || op == OP_I64_MUL_I ||
                      op == OP_I64_AND_I || op == OP_I64_OR_I || op == OP_I64_XOR_I;
      e.sync({a, a + 1, b, b + 1, c, c + 1});
      // operands as word registers; the b operand of *_I in Z
      std::string bl = e.V(b), bh = e.V(b + 1);
      if (ri && op == OP_I64_MUL_I && int32_t(imm) < 0) {   // (the general path below)
        e.l("v_mov_b32 %s, 0x%x", Z0, imm);
        e.l("v_ashrrev_i32_e32 %s, 31, %s", Z1, Z0);
        bl = Z0;
        bh = Z1;
      }
      const std::string al = e.V(a), ah = e.V(a + 1);
      if (ri && op != OP_I64_MUL_I) {
        // a 32-bit immediate (its high word 0 or -1): word by word, straight into the cells
        // unless c overlaps a partly (then through R)
        const bool neg = int32_t(imm) < 0, direct = c == a || c + 1 < a || c > a + 1;
        const std::string lo = direct ? e.V(c) : R0, hi = direct ? e.V(c + 1) : R1;
        if (op == OP_I64_ADD_I) {
          e.l("v_add_co_u32_e32 %s, vcc, 0x%x, %s", lo.c_str(), imm, al.c_str());
          e.l("v_addc_co_u32_e32 %s, vcc, %d, %s, vcc", hi.c_str(), neg ? -1 : 0, ah.c_str());
        } else if (op == OP_I64_SUB_I) {
          e.l("v_subrev_co_u32_e32 %s, vcc, 0x%x, %s", lo.c_str(), imm, al.c_str());
          e.l("v_subbrev_co_u32_e32 %s, vcc, %d, %s, vcc", hi.c_str(), neg ? -1 : 0, ah.c_str());
        } else {
          const bool and_ = op == OP_I64_AND_I, or_ = op == OP_I64_OR_I;
          e.l("%s %s, 0x%x, %s", and_ ? "v_and_b32_e32" : or_ ? "v_or_b32_e32" : "v_xor_b32_e32", lo.c_str(), imm,
              al.c_str());
          if ((and_ && !neg) || (or_ && neg)) e.l("v_mov_b32 %s, %d", hi.c_str(), neg ? -1 : 0);
          else if (!neg || and_ || or_) { if (hi != ah) e.l("v_mov_b32 %s, %s", hi.c_str(), ah.c_str()); }
          else e.l("v_not_b32_e32 %s, %s", hi.c_str(), ah.c_str());
        }
        if (!direct) e.put64(c);
        return true;
      }
      if (op == OP_I64_MUL_I && int32_t(imm) >= 0) {   // (high word 0: no a_lo * b_hi term)
        const bool inl = imm <= 64;
        if (!inl) e.l("s_mov_b32 s68, 0x%x", imm);
        const std::string k = inl ? std::to_string(imm) : std::string("s68");
        e.l("v_mul_hi_u32 %s, %s, %s", X0, al.c_str(), k.c_str());
        e.l("v_mul_lo_u32 %s, %s, %s", Y0, ah.c_str(), k.c_str());
        e.l("v_mul_lo_u32 %s, %s, %s", R0, al.c_str(), k.c_str());
        e.l("v_add_u32_e32 %s, %s, %s", R1, X0, Y0);
        e.put64(c);
        return true;
      }
      if (op == OP_I64_ADD || op == OP_I64_ADD_I) {
        const char *x = e.src64(a, A0, A1, AP);
        const char *y = ri ? ZP : e.src64(b, B0, B1, BP);
        e.l("v_lshl_add_u64 %s, %s, 0, %s", RP, x, y);
      } else if (op == OP_I64_SUB || op == OP_I64_SUB_I) {
        e.l("v_sub_co_u32_e32 %s, vcc, %s, %s", R0, al.c_str(), bl.c_str());
        e.l("v_subb_co_u32_e32 %s, vcc, %s, %s, vcc", R1, ah.c_str(), bh.c_str());
      } else if (op == OP_I64_MUL || op == OP_I64_MUL_I) {
        e.l("v_mul_hi_u32 %s, %s, %s", X0, al.c_str(), bl.c_str());
        e.l("v_mul_lo_u32 %s, %s, %s", X1, al.c_str(), bh.c_str());
        e.l("v_mul_lo_u32 %s, %s, %s", Y0, ah.c_str(), bl.c_str());
        e.l("v_mul_lo_u32 %s, %s, %s", R0, al.c_str(), bl.c_str());
        e.l("v_add3_u32 %s, %s, %s, %s", R1, X0, X1, Y0);
      } else {
        const char *ins = (op == OP_I64_AND || op == OP_I64_AND_I) ? "v_and_b32_e32"
                          : (op == OP_I64_OR || op == OP_I64_OR_I) ? "v_or_b32_e32" : "v_xor_b32_e32";
        e.l("%s %s, %s, %s", ins, R0, al.c_str(), bl.c_str());
        e.l("%s %s, %s, %s", ins, R1, ah.c_str(), bh.c_str());
      }
      e.put64(c);
      return true;
    }
    case OP_I64_SHL: case OP_I64_SHR_S: case OP_I64_SHR_U:
    case OP_I64_SHL_I: case OP_I64_SHR_S_I: case OP_I64_SHR_U_I: {
      const bool ri = op == OP_I64_SHL_I || op == OP_I64_SHR_S_I || op == OP_I64_SHR_U_I;
      const uint16_t base = ri ? uint16_t(op - OP_I64_SHL_I) : uint16_t(op - OP_I64_SHL);
      const char *ins = base == 0 ? "v_lshlrev_b64" : base == 1 ? "v_ashrrev_i64" : "v_lshrrev_b64";
      e.sync({a, a + 1, b, c, c + 1});
      const char *x = e.src64(a, A0, A1, AP);
      const std::string amt = ri ? std::to_string(imm & 63u) : e.V(b);
      e.l("%s %s, %s, %s", ins, RP, amt.c_str(), x);
      e.put64(c);
      return true;
    }
    case OP_I64_ROTL: case OP_I64_ROTR: case OP_I64_ROTL_I: case OP_I64_ROTR_I: {
      const bool left = op == OP_I64_ROTL || op == OP_I64_ROTL_I;
      const bool ri = op == OP_I64_ROTL_I || op == OP_I64_ROTR_I;
      e.sync({a, a + 1, b, c, c + 1});
      const char *x = e.src64(a, A0, A1, AP);
      if (ri) e.l("v_mov_b32 %s, %u", Z0, imm & 63u);
      else e.l("v_mov_b32 %s, %s", Z0, e.v(b));
      e.l("v_sub_u32_e32 %s, 0, %s", Y0, Z0);
      e.l("%s %s, %s, %s", left ? "v_lshlrev_b64" : "v_lshrrev_b64", XP, Z0, x);
      e.l("%s %s, %s, %s", left ? "v_lshrrev_b64" : "v_lshlrev_b64", RP, Y0, x);
      e.l("v_or_b32_e32 %s, %s, %s", R0, R0, X0);
      e.l("v_or_b32_e32 %s, %s, %s", R1, R1, X1);
      e.put64(c);
      return true;
    }
    case OP_I64_EQZ: {
      e.sync({a, a + 1, c});
      const char *x = e.src64(a, A0, A1, AP);
      e.l("v_cmp_eq_u64_e64 vcc, 0, %s", x);
      e.l("v_cndmask_b32_e64 %s, 0, 1, vcc", e.v(c));
      return true;
    }
    case OP_I64_EXTEND_I32_S: case OP_I64_EXT32S:
      e.sync({a, c, c + 1});
      e.l("v_ashrrev_i32_e32 %s, 31, %s", X0, e.v(a));
      if (c != a) e.l("v_mov_b32 %s, %s", e.v(c), e.v(a));
      e.l("v_mov_b32 %s, %s", e.v(c + 1), X0);
      return true;
    case OP_I64_EXTEND_I32_U:
      e.sync({a, c, c + 1});
      if (c != a) e.l("v_mov_b32 %s, %s", e.v(c), e.v(a));
      e.l("v_mov_b32 %s, 0", e.v(c + 1));
      return true;
    case OP_I64_EXT8S: case OP_I64_EXT16S:
      e.sync({a, c, c + 1});
      e.l("v_bfe_i32 %s, %s, 0, %u", R0, e.v(a), op == OP_I64_EXT8S ? 8u : 16u);
      e.l("v_ashrrev_i32_e32 %s, 31, %s", R1, R0);
      e.put64(c);
      return true;
    default:
      break;
  }
  if (mem_bytes(op)) {
    if (is_store_op(op)) return emit_store(e, op, a, b, imm);
    return emit_load(e, op, a, c, imm);
  }
  if (op == OP_XLD || op == OP_XST) return emit_xmem(e, I);
  return false;
}

// ---------------------------------------------------------------- scheduling
// One wave per SIMD (64K instances fill the chip) hides no latency: a VALU instruction
// that needs the result of the one before waits for it (measured: ~12 cycles per
// instruction along a dependent chain against 4 for independent ones). The run's code is
// therefore list-scheduled between barriers (anything but a VALU instruction: scalar
// code, branches, memory, waits), on the registers each instruction names: true, anti
// and output dependences kept, independent chains (BLAKE3's four column / diagonal G
// functions) interleaved.
struct SIns {
  std::string text;
  std::vector<int> defs, uses;
  bool wait = false;   // a counted vmcnt wait: defs = the registers of the loads it retires
  int est = 0;         // (wait) estimated cycle its loads are in
  bool store = false;  // a global store: uses its address and data registers
};

void regs_of(const std::string &tok, std::vector<int> *out) {
  // vN, v[N:M], sN, s[N:M], vcc (VGPR k -> k, SGPR k -> 1000 + k, vcc -> 2000)
  size_t i = 0;
  while (i < tok.size()) {
    const char ch = tok[i];
    const bool word_start = i == 0 || !(isalnum((unsigned char)tok[i - 1]) || tok[i - 1] == '_');
    if (word_start && tok.compare(i, 3, "vcc") == 0) { out->push_back(2000); i += 3; continue; }
    if (word_start && (ch == 'v' || ch == 's') && i + 1 < tok.size()) {
      const int base = ch == 'v' ? 0 : 1000;
      if (tok[i + 1] == '[') {
        int lo = 0, hi = 0;
        if (sscanf(tok.c_str() + i + 2, "%d:%d", &lo, &hi) == 2)
          for (int r = lo; r <= hi; r++) out->push_back(base + r);
        i = tok.find(']', i) + 1;
        continue;
      }
      if (isdigit((unsigned char)tok[i + 1])) {
        out->push_back(base + atoi(tok.c_str() + i + 1));
        i++;
        while (i < tok.size() && isdigit((unsigned char)tok[i])) i++;
        continue;
      }
    }
    i++;
  }
}

bool parse_valu(const std::string &line, SIns *ins) {
  ins->text = line;
  if (line.compare(0, 2, "v_") != 0) return false;
  const size_t sp = line.find(' ');
  if (sp == std::string::npos) return false;
  const std::string mn = line.substr(0, sp);
  std::vector<std::string> ops;
  for (size_t at = sp + 1; at <= line.size();) {
    size_t cm = line.find(", ", at);
    if (cm == std::string::npos) cm = line.size();
    ops.push_back(line.substr(at, cm - at));
    at = cm + 2;
  }
  const size_t ndef = mn.find("_co_") != std::string::npos ? 2 : 1;   // v_add_co: vdst, sdst
  for (size_t k = 0; k < ops.size(); k++) regs_of(ops[k], k < ndef ? &ins->defs : &ins->uses);
  return true;
}

std::string schedule(const std::string &body) {
  std::vector<std::string> lines;
  for (size_t at = 0; at < body.size();) {
    const size_t nl = body.find('\n', at);
    lines.push_back(body.substr(at, nl - at));
    at = nl + 1;
  }
  std::string out;
  std::vector<SIns> seg;
  auto flush = [&]() {
    const size_t n = seg.size();
    if (n > 1) {
      // dependences: j -> i (j earlier) with a latency in cycles
      constexpr int kIssue = 4, kLat = 12;
      std::vector<std::vector<std::pair<int, int>>> pred(n), succ(n);
      std::map<int, int> last_def;
      std::map<int, std::vector<int>> readers;
      int last_wait = -1;
      for (size_t i = 0; i < n; i++) {
        std::map<int, int> dep;   // pred -> latency
        for (int r : seg[i].uses) {
          auto it = last_def.find(r);
          if (it != last_def.end())
            dep[it->second] = std::max(dep[it->second], seg[size_t(it->second)].wait ? 0 : kLat);
        }
        // waits and stores keep their order (the counts are issue-order counts)
        if ((seg[i].wait || seg[i].store) && last_wait >= 0) dep[last_wait] = std::max(dep[last_wait], 0);
        if (seg[i].wait || seg[i].store) last_wait = int(i);
        for (int r : seg[i].defs) {
          auto it = last_def.find(r);
          if (it != last_def.end()) dep[it->second] = std::max(dep[it->second], 1);
          for (int j : readers[r])
            if (j != int(i)) dep[j] = std::max(dep[j], 1);
        }
        for (auto &d : dep) {
          pred[i].push_back({d.first, d.second});
          succ[size_t(d.first)].push_back({int(i), d.second});
        }
        for (int r : seg[i].uses) readers[r].push_back(int(i));
        for (int r : seg[i].defs) { last_def[r] = int(i); readers[r].clear(); }
      }
      std::vector<int> height(n, 0);   // longest latency path to the segment's end
      for (size_t i = n; i-- > 0;)
        for (auto &s : succ[i]) height[i] = std::max(height[i], height[size_t(s.first)] + s.second);
      std::vector<int> npred(n), at(n, 0);
      for (size_t i = 0; i < n; i++) {
        npred[i] = int(pred[i].size());
        if (seg[i].wait) at[i] = seg[i].est;
      }
      std::vector<int> ready;
      for (size_t i = 0; i < n; i++)
        if (!npred[i]) ready.push_back(int(i));
      int clock = 0;
      while (!ready.empty()) {
        size_t best = 0;
        for (size_t k = 1; k < ready.size(); k++) {
          const int a = ready[k], b = ready[best];
          const int ta = std::max(at[size_t(a)], clock), tb = std::max(at[size_t(b)], clock);
          if (ta < tb || (ta == tb && (height[size_t(a)] > height[size_t(b)] ||
                                       (height[size_t(a)] == height[size_t(b)] && a < b))))
            best = k;
        }
        const int i = ready[best];
        ready.erase(ready.begin() + long(best));
        const int t = std::max(at[size_t(i)], clock);
        clock = seg[size_t(i)].wait ? t : t + kIssue;
        out += seg[size_t(i)].text;
        out += '\n';
        for (auto &s : succ[size_t(i)]) {
          at[size_t(s.first)] = std::max(at[size_t(s.first)], t + s.second);
          if (--npred[size_t(s.first)] == 0) ready.push_back(s.first);
        }
      }
    } else if (n == 1) {
      out += seg[0].text;
      out += '\n';
    }
    seg.clear();
  };
  // Counted waits float: the vector-memory operations issued so far (oldest first, the
  // registers each load writes) tell which loads an "s_waitcnt vmcnt(N)" retires; the
  // wait becomes an instruction of the segment that defines those registers, so their
  // readers stay behind it and independent VALU work moves above it. A label whose
  // arrivals may differ (anything but an inlined call's Lpa / a NaN fix's Lnr return)
  // makes the state unknown until the next full wait, and waits then stay barriers.
  constexpr int kLoadLat = 100, kLoadStep = 22;   // cycles: first L2-hit load, each further
  const char *fse = getenv("WB_SCHED_STORES");   // 0: stores stay barriers (A/B aid)
  const bool float_stores = !(fse && fse[0] == '0');
  std::vector<std::vector<int>> vq;   // operations in flight, oldest first
  bool known = true;
  int retired = 0;                    // loads retired by this segment's waits so far
  for (const auto &ln : lines) {
    SIns ins;
    if (parse_valu(ln, &ins)) {
      seg.push_back(std::move(ins));
      continue;
    }
    int nwait = -1;
    if (ln.compare(0, 16, "s_waitcnt vmcnt(") == 0 && ln.find("lgkmcnt") == std::string::npos)
      nwait = atoi(ln.c_str() + 16);
    if (nwait >= 0 && known) {
      SIns w;
      w.text = ln;
      w.wait = true;
      while (vq.size() > size_t(nwait)) {
        for (int r : vq.front()) w.defs.push_back(r);
        vq.erase(vq.begin());
        retired++;
      }
      w.est = kLoadLat + kLoadStep * retired;
      seg.push_back(std::move(w));
      continue;
    }
    if (ln.compare(0, 12, "global_store") == 0 && known && float_stores) {
      // a store only reads registers: VALU work moves across it (its data and address
      // registers' writers stay before it, later writers after it)
      SIns st;
      st.text = ln;
      st.store = true;
      const size_t sp = ln.find(' ');
      if (sp != std::string::npos) regs_of(ln.substr(sp + 1), &st.uses);
      seg.push_back(std::move(st));
      vq.push_back({});
      continue;
    }
    flush();
    retired = 0;
    out += ln;
    out += '\n';
    if (ln.compare(0, 11, "global_load") == 0) {
      std::vector<int> d;
      const size_t sp = ln.find(' '), cm = ln.find(',');
      if (sp != std::string::npos && cm != std::string::npos) regs_of(ln.substr(sp + 1, cm - sp - 1), &d);
      vq.push_back(d);
    } else if (ln.compare(0, 7, "global_") == 0 || ln.compare(0, 7, "buffer_") == 0) {
      vq.push_back({});
    } else if (ln.find("vmcnt(0)") != std::string::npos) {
      vq.clear();
      known = true;
    } else if (!ln.empty() && ln.back() == ':' && ln.compare(0, 3, "Lpa") != 0 &&
               ln.compare(0, 3, "Lnr") != 0) {
      known = false;
    }
  }
  flush();
  return out;
}

// cells an instruction writes (for the access groups: a write to the address cell ends
// its group)
void written(const DInstr &I, std::vector<uint32_t> *out) {
  const uint16_t op = op_of(I);
  const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16, c = I.w2 & 0xFFFFu, d = I.w2 >> 16;
  out->clear();
  if (is_store_op(op) || op == OP_NOP_CNT || op == OP_XST) return;
  if (op == OP_ZERO_LOCALS) {
    for (uint32_t k = 0; k < b; k++) out->push_back(a + k);
    return;
  }
  for (uint32_t k = 0; k < 4; k++) out->push_back(c + k);   // (over-approximates narrower results)
  if (op == OP_I32_ADD_XROTR_I) out->push_back(d);
  if (op == OP_I32_ADD3_XROTR_I) out->push_back(I.w3 & 0xFFFFu);
}

// The access groups of a run (see "linear memory"): lead[i] = group index of the access
// at pc + i that checks its group, -1 otherwise.
std::vector<MemGroup> jit_groups(const Program &P, const JitRun &r, std::vector<int> *lead) {
  std::vector<MemGroup> G;
  lead->assign(r.len, -1);
  int open = -1;
  std::vector<uint32_t> wr;
  for (uint32_t i = 0; i < r.len; i++) {
    const DInstr &I = P.code[r.pc + i];
    const uint16_t op = op_of(I);
    if (xmop(I)) open = -1;   // (an extra memory's access computes its address in the temps)
    if (const uint32_t n = mem_bytes(op)) {
      const uint32_t a = I.w1 & 0xFFFFu, imm = I.w3;
      if (open < 0 || G[size_t(open)].base != a) {
        open = int(G.size());
        G.emplace_back();
        G.back().base = a;
        (*lead)[i] = open;
      }
      MemGroup &g = G[size_t(open)];
      g.maxlast = std::max(g.maxlast, imm + n - 1);
      if (is_store_op(op))
        g.store_end = std::max<uint64_t>(g.store_end, uint64_t(imm) + n);
      const uint32_t m = n >= 4 ? 3 : n - 1;
      if (m) {
        const std::pair<uint32_t, uint32_t> am{imm & m, m};
        if (std::find(g.aligns.begin(), g.aligns.end(), am) == g.aligns.end()) g.aligns.push_back(am);
      }
    }
    written(I, &wr);
    if (open >= 0 && std::find(wr.begin(), wr.end(), G[size_t(open)].base) != wr.end()) open = -1;
  }
  return G;
}

// Load batches: a run's consecutive loads (BLAKE3's 16 message and 8 chaining words) are
// issued in the order the rest of the run first needs them, so that counted waits
// (Em::sync) let the first uses start while later words still stream in (one wave per
// SIMD: each further L2-hit load waited for costs ~22 cycles, MI355X_MICROARCH.md).
// Every group of the batch is checked first; a failing check leaves before the batch's
// first load (nothing of the batch has happened yet, and the C++ step or the handlers
// then meet the failing access in program order). A batch is at most two groups (base
// pairs v[122:123], v[124:125]) and no load of it writes a cell another one reads or
// writes.
struct LoadBatch {
  uint32_t i0 = 0, i1 = 0;       // run body indices [i0, i1)
  std::vector<uint32_t> order;   // issue order (body indices)
};

bool load_wide(uint16_t op) { return load_wide_op(op); }
uint32_t load_cells(uint16_t op) { return op == OP_LD128 ? 4u : load_wide(op) ? 2u : 1u; }

// an operand field naming the cell (or the cell below it: a 64-bit operand's high word);
// only the batch's issue order depends on it
bool mentions(const DInstr &I, uint32_t cell) {
  const uint32_t f[5] = {I.w1 & 0xFFFFu, I.w1 >> 16, I.w2 & 0xFFFFu, I.w2 >> 16,
                         op_of(I) == OP_I32_ADD3_XROTR_I ? (I.w3 & 0xFFFFu) : 0xFFFFu};
  for (uint32_t x : f)
    if (x != 0xFFFFu && (cell == x || cell == x + 1)) return true;
  return false;
}

std::vector<LoadBatch> load_batches(const Program &P, const JitRun &r, uint32_t nbody,
                                    const std::vector<int> &lead) {
  std::vector<LoadBatch> out;
  auto is_load = [&](uint32_t i) {
    const uint16_t op = op_of(P.code[r.pc + i]);
    return mem_bytes(op) && !is_store_op(op);
  };
  for (uint32_t i = 0; i < nbody;) {
    if (!is_load(i) || lead[i] < 0) { i++; continue; }
    std::vector<uint32_t> addr, dest;
    uint32_t j = i, leads = 0;
    for (; j < nbody && is_load(j); j++) {
      const DInstr &I = P.code[r.pc + j];
      const uint32_t a = I.w1 & 0xFFFFu, c = I.w2 & 0xFFFFu, nc = load_cells(op_of(I));
      if (lead[j] >= 0 && ++leads > 2) break;
      bool clash = std::find(dest.begin(), dest.end(), a) != dest.end();
      for (uint32_t q = 0; q < nc; q++)
        clash = clash || std::find(dest.begin(), dest.end(), c + q) != dest.end() ||
                std::find(addr.begin(), addr.end(), c + q) != addr.end();
      if (clash) break;
      addr.push_back(a);
      for (uint32_t q = 0; q < nc; q++) dest.push_back(c + q);
    }
    if (j - i >= 2) {
      LoadBatch b;
      b.i0 = i;
      b.i1 = j;
      std::vector<std::pair<uint32_t, uint32_t>> key;   // (first use, index)
      for (uint32_t k = i; k < j; k++) {
        const DInstr &I = P.code[r.pc + k];
        const uint32_t c = I.w2 & 0xFFFFu, nc = load_cells(op_of(I));
        uint32_t t = j;
        for (; t < r.len; t++) {
          bool m = false;
          for (uint32_t q = 0; q < nc; q++) m = m || mentions(P.code[r.pc + t], c + q);
          if (m) break;
        }
        key.push_back({t, k});
      }
      std::stable_sort(key.begin(), key.end(),
                       [](const std::pair<uint32_t, uint32_t> &x, const std::pair<uint32_t, uint32_t> &y) {
                         return x.first < y.first;
                       });
      for (auto &kv : key) b.order.push_back(kv.second);
      out.push_back(std::move(b));
    }
    i = j;
  }
  return out;
}

bool emit(Em &e, const DInstr &I);

// the batch's checks (leaving before its first load), then its loads in issue order
void emit_batch(Em &e, const Program &P, uint32_t rpc, const LoadBatch &b,
                const std::vector<MemGroup> &G, const std::vector<int> &lead) {
  std::vector<uint32_t> bv(b.i1 - b.i0, 122);
  uint32_t groups = 0;
  e.pc = rpc + b.i0;
  for (uint32_t k = b.i0; k < b.i1; k++) {
    if (lead[k] >= 0) {
      e.basev = groups++ ? 124 : 122;
      group_check(e, G[size_t(lead[k])]);
    }
    bv[k - b.i0] = e.basev;
  }
  e.group = nullptr;
  for (uint32_t k : b.order) {
    e.pc = rpc + k;
    e.basev = bv[k - b.i0];
    emit(e, P.code[rpc + k]);
  }
  e.basev = bv.back();   // (the group still open after the batch)
  e.pc = rpc + b.i1 - 1;
}

// CALL (gen_tc.py call_body_v): spill [fb, L) and the return record to the LDS call
// stack, args L.. -> fb.., zero the callee's locals, jump to the callee.
// Zeroing a callee local is dead when the callee's first compiled run writes it before
// anything could read it: on every path from the body start the run's instructions come
// first in program order (the interpreter resumes a run that leaves mid-way at the same
// instruction), so the zero is never observed. Writes are taken only from instructions
// whose destination is certain; any operand field that names the cell counts as a read.
bool is_xfer(uint16_t op);
bool is_branch_op(uint16_t op);
std::vector<uint8_t> dead_zeros(const Program &P, const JitRun &r) {
  std::vector<uint8_t> dead(TC_VF_CELLS, 0), seen(TC_VF_CELLS, 0);
  for (uint32_t i = 0; i < r.len; i++) {
    const DInstr &I = P.code[r.pc + i];
    const uint16_t op = op_of(I);
    const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16, c = I.w2 & 0xFFFFu, d = I.w2 >> 16;
    auto rd = [&](uint32_t x, uint32_t n) {
      for (uint32_t k = 0; k < n; k++)
        if (x + k < TC_VF_CELLS) seen[x + k] = 1;
    };
    rd(a, 4); rd(b, 4); rd(d, 4);
    if (op == OP_I32_ADD3_XROTR_I) rd(I.w3 & 0xFFFFu, 1);
    if (op == OP_ZERO_LOCALS || op == OP_POST_CALL || is_xfer(op) || is_branch_op(op)) {
      rd(0, TC_VF_CELLS);   // (no claims past these)
      continue;
    }
    uint32_t w = 0;   // certain 32-bit words written at c
    switch (op) {
      case OP_LD32: case OP_LD8S32: case OP_LD8U32: case OP_LD16S32: case OP_LD16U32:
      case OP_CONST32: case OP_MOV32: case OP_I32_ADD: case OP_I32_SUB: case OP_I32_MUL:
      case OP_I32_AND: case OP_I32_OR: case OP_I32_XOR: case OP_I32_ADD_I: case OP_I32_SUB_I:
      case OP_I32_AND_I: case OP_I32_OR_I: case OP_I32_XOR_I: case OP_I32_SHL_I:
      case OP_I32_SHR_U_I: case OP_I32_SHR_S_I:
        w = 1; break;
      case OP_CONST64: case OP_MOV64: case OP_LD64: case OP_LD32U64: case OP_LD32S64:
        w = 2; break;
      default: break;
    }
    for (uint32_t k = 0; k < w; k++)
      if (c + k < TC_VF_CELLS && !seen[c + k]) dead[c + k] = 1;
    rd(c, w ? w : 4);
  }
  return dead;
}

void emit_call(Em &e, const DInstr &I, uint32_t pc, const std::vector<uint8_t> *dead) {
  const uint32_t L = I.w1 & 0xFFFFu, nargs = I.w1 >> 16, nloc = I.w2 & 0xFFFFu, fb = e.fb;
  const uint32_t n = L - fb;
  if (!e.call_checked) {
    e.l("v_add_u32_e32 %s, %u, v102", X0, n + 1);
    e.l("v_cmp_lt_u32_e64 %s, s93, %s", T2, X0);   // would pass the LDS part: the C++ step
    e.leave_if_t2();
  }
  e.l("v_lshl_add_u32 %s, v102, 8, v103", X1);
  for (uint32_t k = 0; k < n; k++) e.l("ds_write_b32 %s, %s offset:%u", X1, e.v(fb + k), k * 256u);
  e.l("v_mov_b32 %s, 0x%x", Y1, ((pc + 1) & 0xFFFFFu) | (L << 20));
  e.l("ds_write_b32 %s, %s offset:%u", X1, Y1, n * 256u);
  e.l("v_add_u32_e32 v102, %u, v102", n + 1);
  for (uint32_t k = 0; k < nargs; k++)
    if (L != fb) e.l("v_mov_b32 %s, %s", e.v(fb + k), e.v(L + k));
  for (uint32_t k = 0; k < nloc; k++)
    if (!dead || !(*dead)[fb + nargs + k]) e.l("v_mov_b32 %s, 0", e.v(fb + nargs + k));
}

// TAIL_CALL (return_call, dbc_step.inc OP_TAIL_CALL; gen_tc.py tail_call_body): the
// callee takes over the frame -- arguments L.. -> fb.. (ascending: L >= fb), its live
// locals zeroed; no spill, no return record, then the transfer to its body like a jump.
void emit_tail_call(Em &e, const DInstr &I, const std::vector<uint8_t> *dead) {
  const uint32_t L = I.w1 & 0xFFFFu, nargs = I.w1 >> 16, nloc = I.w2 & 0xFFFFu, fb = e.fb;
  for (uint32_t k = 0; k < nargs; k++)
    if (L != fb) e.l("v_mov_b32 %s, %s", e.v(fb + k), e.v(L + k));
  for (uint32_t k = 0; k < nloc; k++)
    if (!dead || !(*dead)[fb + nargs + k]) e.l("v_mov_b32 %s, 0", e.v(fb + nargs + k));
}

// RET (gen_tc.py ret_body_v): pop the return record (it must agree across the lanes and
// not be the entry frame's), results a.. -> fb.., jump to the return pc.
// split: (SIMT) where the lanes' return records disagree, go there (Y1 = the records);
// else leave before the return. Returns the leave stub's label.
// One test decides the common case: a lane whose call stack reaches past its LDS part
// reads its record as ~0 (an entry-frame record: it leaves), and an entry-frame record in
// the first lane counts as a disagreement, so a single branch takes every exception to
// `split` (which leaves for entry-frame records) or to the leave stub. (An LDS read past
// the allocation returns 0 and cannot fault; the record of such a lane is discarded.)
// known: up to two (return record, label) pairs: where every lane's record is the same
// known one the group goes straight to that label (the records of a function's direct call
// sites are constants), before the agreement test.
std::string emit_ret(Em &e, const DInstr &I, const std::string &split,
                     const std::vector<std::pair<uint32_t, std::string>> &known = {}) {
  const uint32_t a = I.w1 & 0xFFFFu, nres = I.w1 >> 16, fb = e.fb;
  const std::string out = e.leave_stub();
  if (e.ret_pf_done && e.stack_ok) {
    e.l("v_mov_b32 %s, v113", Y1);
  } else if (e.ret_pf_done) {
    e.l("v_cmp_lt_u32_e32 vcc, s93, v102");
    e.l("v_cndmask_b32_e64 %s, v113, -1, vcc", Y1);
  } else {
    e.l("v_lshl_add_u32 %s, v102, 8, v103", X1);
    e.l("v_subrev_u32_e32 %s, 0x100, %s", X1, X1);
    e.l("ds_read_b32 %s, %s", Y1, X1);
    e.l("v_cmp_lt_u32_e32 vcc, s93, v102");
    e.l("s_waitcnt lgkmcnt(0)");
    e.l("v_cndmask_b32_e64 %s, %s, -1, vcc", Y1, Y1);
  }
  if (!known.empty()) {
    if (known.size() > 1) e.l("v_mov_b32 %s, 0x%x", X0, known[1].first);
    e.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", known[0].first, Y1);
    if (known.size() > 1) e.l("v_cmp_eq_u32_e64 s[68:69], %s, %s", X0, Y1);
    e.l("s_and_b64 vcc, vcc, exec");
    e.l("s_cmp_eq_u64 vcc, exec");
    e.l("s_cbranch_scc1 %s", known[0].second.c_str());
    if (known.size() > 1) {
      e.l("s_and_b64 s[68:69], s[68:69], exec");
      e.l("s_cmp_eq_u64 s[68:69], exec");
      e.l("s_cbranch_scc1 %s", known[1].second.c_str());
    }
  }
  e.l("v_readfirstlane_b32 s68, %s", Y1);
  e.l("s_nop 1");
  e.l("v_cmp_ne_u32_e64 %s, s68, %s", T2, Y1);
  e.l("s_and_b32 s68, s68, 0xfffff");
  e.l("s_cmp_eq_u32 s68, 0xfffff");
  e.l("s_cselect_b64 %s, exec, %s", T2, T2);
  e.l("s_and_b64 %s, %s, exec", T2, T2);
  e.l("s_cbranch_scc1 %s", split.empty() ? out.c_str() : split.c_str());
  e.l("v_subrev_u32_e32 v102, 1, v102");
  for (uint32_t k = 0; k < nres; k++)
    if (a != fb) e.l("v_mov_b32 %s, %s", e.v(fb + k), e.v(a + k));
  e.l("s_lshl_b32 s62, s68, 5");
  return out;
}

// BR_TABLE (controlInstr.cpp:53-70; dbc_step.inc): index = min(cell a, b) (b = the
// default's index), entry brtab[imm + index] = (target pc, taken-count correction).
// Per lane: Y0 = target, Y1 = correction. A table of at most 4 entries whose targets fit a
// byte and corrections a signed byte (C4's state machine) reads both as byte fields of a
// constant (v_bfe at 8 * index); larger ones take a compare chain over the entries that
// differ from the default, with inline constants where they fit.
void emit_br_table(Em &e, const DInstr &I) {
  const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16, imm = I.w3;
  const std::vector<uint32_t> &bt = e.prog->brtab;
  auto tgt = [&](uint32_t k) { return bt[2 * (imm + k)]; };
  auto cor = [&](uint32_t k) { return int32_t(bt[2 * (imm + k) + 1]); };
  bool same_c = true, bytes = b < 4;
  for (uint32_t k = 0; k <= b; k++) {
    same_c = same_c && cor(k) == cor(b);
    bytes = bytes && tgt(k) < 256 && cor(k) >= -128 && cor(k) <= 127;
  }
  e.l("v_min_u32_e32 %s, 0x%x, %s", X0, b, e.v(a));
  if (bytes) {
    uint32_t kt = 0, kc = 0;
    for (uint32_t k = 0; k <= b; k++) {
      kt |= tgt(k) << (8 * k);
      kc |= (uint32_t(cor(k)) & 0xFFu) << (8 * k);
    }
    e.l("v_lshlrev_b32_e32 %s, 3, %s", X1, X0);
    e.l("v_mov_b32 %s, 0x%x", Y0, kt);
    e.l("v_bfe_u32 %s, %s, %s, 8", Y0, Y0, X1);
    if (same_c) {
      e.l("v_mov_b32 %s, 0x%x", Y1, uint32_t(cor(b)));
    } else {
      e.l("v_mov_b32 %s, 0x%x", Y1, kc);
      e.l("v_bfe_i32 %s, %s, %s, 8", Y1, Y1, X1);
    }
    return;
  }
  auto inl = [](uint32_t v) { return int32_t(v) >= -16 && int32_t(v) <= 64; };
  auto sel = [&](const char *dst, uint32_t v) {   // dst = vcc ? v : dst
    if (inl(v)) {
      e.l("v_cndmask_b32_e64 %s, %s, %d, vcc", dst, dst, int32_t(v));
    } else {
      e.l("v_mov_b32 %s, 0x%x", X1, v);
      e.l("v_cndmask_b32_e32 %s, %s, %s, vcc", dst, dst, X1);
    }
  };
  e.l("v_mov_b32 %s, 0x%x", Y0, tgt(b));
  e.l("v_mov_b32 %s, 0x%x", Y1, uint32_t(cor(b)));
  for (uint32_t k = 0; k < b; k++) {
    if (tgt(k) == tgt(b) && cor(k) == cor(b)) continue;
    e.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", k, X0);
    if (tgt(k) != tgt(b)) sel(Y0, tgt(k));
    if (cor(k) != cor(b)) sel(Y1, uint32_t(cor(k)));
  }
}

// can instruction I be compiled (dry run)
bool jit_ok(const Program &P, const DInstr &I) {
  const uint16_t op = op_of(I);
  if (const uint32_t n = mem_bytes(op))
    if (uint64_t(I.w3) + n - 1 > 0xFFFFFFFFull) return false;
  Em e;
  e.fb = P.global_cells;
  e.prog = &P;
  return emit(e, I);
}

}  // namespace

uint64_t JitCost::full(const Program &P, uint32_t pc) const {
  const uint32_t cnt = (P.code[pc].w0 >> 16) & 0xFFu;
  return cnt ? (*pool)[(*off)[pc] + cnt - 1] : 0;
}

int64_t JitCost::taken(uint32_t to, int32_t jtc) const {
  if (jtc < 0) return -int64_t((*pool)[(*off)[to] + uint32_t(-jtc) - 1u]);
  return int64_t(c_else) * jtc;
}

namespace {

bool is_xfer(uint16_t op) { return op == OP_CALL || op == OP_RET; }
bool is_branch_op(uint16_t op) {
  return op == OP_JMP || op == OP_BR_IF || op == OP_BR_UNLESS || (op >= OP_BR_EQ && op <= OP_BR_GE_U_I);
}
bool ends_run(uint16_t op) { return is_xfer(op) || is_branch_op(op) || op == OP_BR_TABLE || op == OP_TAIL_CALL; }


// The compare of a branch into vcc (true = taken).
void branch_cond(Em &e, const DInstr &I) {
  const uint16_t op = op_of(I);
  const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16;
  if (op == OP_BR_IF) {
    e.l("v_cmp_ne_u32_e32 vcc, 0, %s", e.v(a));
  } else if (op == OP_BR_UNLESS) {
    e.l("v_cmp_eq_u32_e32 vcc, 0, %s", e.v(a));
  } else if (op >= OP_BR_EQ_I) {   // b: a signed imm16
    const uint16_t k = uint16_t(op - OP_BR_EQ_I);
    e.l("v_cmp_%s32_e32 vcc, %d, %s", cmp_kind(cmp_swap(k)), int32_t(int16_t(b)), e.v(a));
  } else {
    const uint16_t k = uint16_t(op - OP_BR_EQ);
    e.l("v_cmp_%s32_e32 vcc, %s, %s", cmp_kind(k), e.v(a), e.v(b));
  }
}

}  // namespace

std::vector<JitRun> jit_runs(const Program &P, const std::vector<TInstr> &tc, bool simt, bool trip) {
  std::vector<JitRun> runs;
  const size_t n = P.code.size();
  if (P.total_cells() > TC_VF_CELLS) return runs;
  const std::vector<uint8_t> target = jump_targets(P);
  std::vector<uint8_t> ok(n, 0);
  (void)tc;
  // (br_table only with SIMT: its splits stay in the core, and SIMT contexts are never
  // metered, whose compiled runs would have to price each table entry)
  for (size_t pc = 0; pc < n; pc++)
    ok[pc] = jit_ok(P, P.code[pc]) && (simt || op_of(P.code[pc]) != OP_BR_TABLE) &&
             (op_of(P.code[pc]) != OP_TAIL_CALL || (simt && !trip));   // (SIMT transfers only)
  for (size_t pc = 0; pc < n;) {
    if (!ok[pc]) { pc++; continue; }
    // a run ends after a call, return or branch (the run's code makes the transfer)
    size_t end = pc + 1;
    if (!ends_run(op_of(P.code[pc])))
      while (end < n && ok[end] && !target[end] && end - pc < kMaxRun) {
        end++;
        if (ends_run(op_of(P.code[end - 1]))) break;
      }
    bool calls = false;   // the call protocol's handlers are long: worth a run of any length
    for (size_t k = pc; k < end; k++) {
      const uint16_t o = op_of(P.code[k]);
      calls |= is_xfer(o) || o == OP_POST_CALL || o == OP_BR_TABLE || o == OP_TAIL_CALL;
    }
    // a lone branch: only with SIMT, where its splits then stay in the core
    if (end - pc == 1 && is_branch_op(op_of(P.code[pc]))) calls = simt && op_of(P.code[pc]) != OP_JMP;
    // (trip mode: every compilable stretch, or its lanes would wait outside the trips)
    if (end - pc >= kMinRun || calls || (trip && simt)) {
      uint32_t cnt = 0;
      for (size_t k = pc; k < end; k++) cnt += (P.code[k].w0 >> 16) & 0xFFu;
      runs.push_back(JitRun{uint32_t(pc), uint32_t(end - pc), cnt});
    }
    pc = end;
  }
  return runs;
}

// ---------------------------------------------------------------- SIMT scheduling
// (KParams::simt) Every running lane of the wave is in the core: ALL = s[96:97], their
// frames in v128.. . The group in EXEC runs at PCOFF; every other lane in ALL waits at its
// own pc in VPC (v92). VCNT (v93) holds each lane's retired instructions not yet counted
// in CNT (s65), which only the group advances. Where the group's lanes part ways (a split
// branch or return) or it reaches OTHER (the lowest waiting pc: lanes merge there), it
// records its lanes' pcs and counts (a "flush": CNT moves into VCNT and comes off the
// budget LIM) and Lsched picks the next group: the lanes at the lowest pc (min-pc
// reconvergence, as the kernel's scheduler), OTHER/LOW = the lowest pc of the rest, the
// handler banks of the matching mode (converged C / diverged D: gen_tc.py), and
// dispatches its TInstr. Lanes never leave the core here; the core returns to the kernel
// (the group's next instruction in the C++ step, or LIM spent) with VPC/VCNT for all.
const char *const VPC = "v92", *const VCNT = "v93";

// CNT into VCNT for the group, off the budget LIM
void flush(Em &e) {
  e.l("v_add_u32_e32 %s, s65, %s", VCNT, VCNT);
  e.l("s_sub_u32 s64, s64, s65");
  e.l("s_cselect_b32 s64, 0, s64");
  e.l("s_mov_b32 s65, 0");
}

// jump to label `to` from anywhere in the code object: a placeholder that resolve_jumps
// turns into s_branch when the target is surely within its +-128 KiB, else into a
// pc-relative s_setpc through s[68:69]
void long_jump(Em &e, const std::string &to, const std::string &tag) {
  e.l("LJMP %s %s", to.c_str(), tag.c_str());
}

// conditional form: to label `to` when SCC is 1 (s_cbranch_scc1 when near, else around
// a long jump)
void cond_jump(Em &e, const std::string &to, const std::string &tag) {
  e.l("LJCC %s %s", to.c_str(), tag.c_str());
}

std::string resolve_jumps(const std::string &body) {
  std::vector<std::string> lines;
  for (size_t at = 0; at < body.size();) {
    size_t nl = body.find('\n', at);
    if (nl == std::string::npos) nl = body.size();
    lines.push_back(body.substr(at, nl - at));
    at = nl + 1;
  }
  // an upper bound on the bytes before each line: 12 per instruction (8 + a literal),
  // 64 per alignment
  std::vector<uint64_t> pos(lines.size() + 1, 0);
  std::map<std::string, size_t> lab;
  for (size_t i = 0; i < lines.size(); i++) {
    const std::string &ln = lines[i];
    uint64_t b = 12;
    if (ln.empty() || ln[0] == '.') b = ln.compare(0, 8, ".p2align") == 0 ? 64 : 0;
    if (ln.compare(0, 5, "LJMP ") == 0 || ln.compare(0, 5, "LJCC ") == 0) b = 48;   // (the long form)
    if (!ln.empty() && ln.back() == ':') { lab[ln.substr(0, ln.size() - 1)] = i; b = 0; }
    pos[i + 1] = pos[i] + b;
  }
  std::string out;
  out.reserve(body.size() + body.size() / 4);
  for (size_t i = 0; i < lines.size(); i++) {
    const std::string &ln = lines[i];
    const bool cc = ln.compare(0, 5, "LJCC ") == 0;
    if (ln.compare(0, 5, "LJMP ") != 0 && !cc) { out += ln; out += '\n'; continue; }
    const size_t sp = ln.find(' ', 5);
    const std::string to = ln.substr(5, sp - 5), tag = ln.substr(sp + 1);
    auto it = lab.find(to);
    const uint64_t d = it == lab.end() ? ~0ull
                                       : (pos[it->second] > pos[i] ? pos[it->second] - pos[i]
                                                                    : pos[i] - pos[it->second]);
    if (d < 100000) {
      out += (cc ? "s_cbranch_scc1 " : "s_branch ") + to + "\n";
    } else if (cc) {
      out += "s_cbranch_scc0 " + tag + "_n\n";
      out += "s_getpc_b64 s[68:69]\n" + tag + ":\n";
      out += "s_add_u32 s68, s68, " + to + " - " + tag + "\n";
      out += "s_addc_u32 s69, s69, (" + to + " - " + tag + ") >> 32\n";
      out += "s_setpc_b64 s[68:69]\n" + tag + "_n:\n";
    } else {
      out += "s_getpc_b64 s[68:69]\n" + tag + ":\n";
      out += "s_add_u32 s68, s68, " + to + " - " + tag + "\n";
      out += "s_addc_u32 s69, s69, (" + to + " - " + tag + ") >> 32\n";
      out += "s_setpc_b64 s[68:69]\n";
    }
  }
  return out;
}

// min over the lanes of `mask` (an SGPR pair) of VPC into SGPR `dst` (~0 when none);
// EXEC = all 64 lanes on entry and exit
void wave_min_of(Em &e, const char *mask, const char *src, const char *dst) {
  e.l("v_cndmask_b32_e64 %s, -1, %s, %s", X0, src, mask);
  static const char *const steps[6] = {"row_shr:1 row_mask:0xf", "row_shr:2 row_mask:0xf",
                                       "row_shr:4 row_mask:0xf", "row_shr:8 row_mask:0xf",
                                       "row_bcast:15 row_mask:0xa", "row_bcast:31 row_mask:0xc"};
  for (const char *st : steps) {
    e.l("s_nop 1");
    e.l("v_min_u32_dpp %s, %s, %s %s bank_mask:0xf", X0, X0, X0, st);
  }
  e.l("s_nop 1");
  e.l("v_readlane_b32 %s, %s, 63", dst, X0);
  e.l("s_nop 1");
}
void wave_min_vpc(Em &e, const char *mask, const char *dst) { wave_min_of(e, mask, VPC, dst); }

// The scheduler's pick: the lanes of `mask` (ALL, or another SGPR pair: trip mode's
// lanes outside the trips) at their lowest pc are the group, OTHER/LOW = the lowest pc of
// the other lanes in ALL, the handler banks of the matching mode, and the group's TInstr
// is dispatched. `p`: label prefix (Lsc for Lsched).
void sched_block(Em &e, const std::string &p, const char *mask, bool depth = false) {
  // every pick costs 16 of the budget as well: the core returns to the kernel (limits,
  // interrupts) even if the lanes retired nothing
  e.l("s_sub_u32 s64, s64, 16");
  e.l("s_cselect_b32 s64, 0, s64");
  if (!mask && depth) {
    // Recursive modules (jit_source: depth_pick): the group is every lane at the pc of the
    // lane lowest in its call stack (fewest stack slots; ties: the lowest pc). LOW = the
    // lowest waiting pc, OTHER = the lowest waiting pc above the group's (= LOW when the
    // group is the lowest): the group runs on until it reaches OTHER or jumps to or below
    // LOW, so it follows its lanes' calls and returns past lanes waiting lower in the
    // function instead of stopping at them -- lanes in different parts of their call trees
    // meet at the pcs where the others wait (C1: 1.43 -> 1.04 group runs per run of the
    // slowest lane in a model of its traces, tools/fib_probe.py)
    e.l("s_mov_b64 exec, -1");
    e.l("s_waitcnt lgkmcnt(0)");   // (a TInstr prefetch must land: s[76:77] is a temp here)
    e.l("s_nop 4");
    e.l("v_min_u32_e32 %s, 0xfff, v102", X1);
    e.l("v_lshl_or_b32 %s, %s, 20, %s", X1, X1, VPC);
    e.l("s_nop 1");
    wave_min_of(e, "s[96:97]", X1, "s68");
    e.l("s_and_b32 s68, s68, 0xfffff");                  // the group's pc
    e.l("s_lshl_b32 s62, s68, 5");
    e.l("v_cmp_eq_u32_e64 s[74:75], s68, %s", VPC);
    e.l("s_and_b64 s[74:75], s[74:75], s[96:97]");       // the group: ALL at that pc
    e.l("s_cmp_eq_u32 s95, -1");                         // were the banks converged?
    e.l("s_cselect_b32 s69, 1, 0");
    e.l("s_andn2_b64 vcc, s[96:97], s[74:75]");          // the lanes left waiting
    e.l("s_cbranch_vccz %s_conv", p.c_str());
    wave_min_vpc(e, "vcc", "s63");                       // LOW (a pc)
    e.l("s_cmp_gt_u32 s63, s68");
    e.l("s_cbranch_scc1 %s_ol", p.c_str());
    e.l("s_lshl_b32 s95, s63, 5");
    e.l("v_cmp_lt_u32_e64 s[76:77], s68, %s", VPC);
    e.l("s_and_b64 s[76:77], s[76:77], vcc");            // waiting above the group's pc
    wave_min_vpc(e, "s[76:77]", "s63");                  // OTHER (~0: none)
    e.l("s_cmp_eq_u32 s63, -1");
    e.l("s_cbranch_scc1 %s_od", p.c_str());
    e.l("s_lshl_b32 s63, s63, 5");
    e.l("s_branch %s_od", p.c_str());
    e.l("%s_ol:", p.c_str());
    e.l("s_lshl_b32 s63, s63, 5");
    e.l("s_mov_b32 s95, s63");
    e.l("%s_od:", p.c_str());
    e.l("s_waitcnt lgkmcnt(0)");
    e.l("s_load_dwordx8 s[76:83], s[60:61], s62");
    e.l("s_load_dwordx8 s[84:91], s[60:61], s62 offset:0x20");
    e.l("s_cmp_eq_u32 s69, 0");
    e.l("s_cbranch_scc1 %s_disp", p.c_str());
    e.l("s_add_u32 s70, s70, 0x%x", 2u * TC_BANK_BYTES);  // C -> D banks
    e.l("s_addc_u32 s71, s71, 0");
    e.l("s_branch %s_bankb", p.c_str());
    e.l("%s_conv:", p.c_str());
    e.l("s_waitcnt lgkmcnt(0)");
    e.l("s_load_dwordx8 s[76:83], s[60:61], s62");
    e.l("s_load_dwordx8 s[84:91], s[60:61], s62 offset:0x20");
    e.l("s_mov_b32 s63, -1");
    e.l("s_mov_b32 s95, -1");
    e.l("s_cmp_eq_u32 s69, 1");
    e.l("s_cbranch_scc1 %s_disp", p.c_str());
    e.l("s_sub_u32 s70, s70, 0x%x", 2u * TC_BANK_BYTES);  // D -> C banks
    e.l("s_subb_u32 s71, s71, 0");
    e.l("%s_bankb:", p.c_str());
    e.l("s_add_u32 s72, s70, 0x%x", TC_BANK_BYTES);
    e.l("s_addc_u32 s73, s71, 0");
    e.l("%s_disp:", p.c_str());
    e.l("s_mov_b64 exec, s[74:75]");
    e.l("s_cmp_eq_u32 s64, 0");                          // budget spent: to the kernel
    e.l("s_cbranch_scc1 %s_out", p.c_str());
    e.l("s_waitcnt lgkmcnt(0)");
    e.l("s_add_u32 s68, s70, s76");
    e.l("s_addc_u32 s69, s71, 0");
    e.l("s_setpc_b64 s[68:69]");
    e.l("%s_out:", p.c_str());
    e.l("s_add_u32 s68, s70, %u", TC_JIT_XS);
    e.l("s_addc_u32 s69, s71, 0");
    e.l("s_setpc_b64 s[68:69]");
    return;
  }
  e.l("s_mov_b64 exec, -1");
  if (mask) e.l("s_mov_b64 s[74:75], %s", mask);   // (the TInstr load below overwrites s[76:91])
  e.l("s_nop 4");
  wave_min_vpc(e, mask ? "s[74:75]" : "s[96:97]", "s68");   // the lowest pc
  e.l("s_lshl_b32 s62, s68, 5");
  // the group's TInstr loads while the rest of the pick goes on (a prefetch still in
  // flight must land first: SMEM returns out of order)
  e.l("s_waitcnt lgkmcnt(0)");
  e.l("s_load_dwordx8 s[76:83], s[60:61], s62");
  e.l("s_load_dwordx8 s[84:91], s[60:61], s62 offset:0x20");
  if (mask) {
    e.l("v_cmp_eq_u32_e64 vcc, s68, %s", VPC);
    e.l("s_and_b64 s[74:75], vcc, s[74:75]");          // the group: the mask's lanes at that pc
  } else {
    e.l("v_cmp_eq_u32_e64 s[74:75], s68, %s", VPC);
    e.l("s_and_b64 s[74:75], s[74:75], s[96:97]");     // the group: ALL at that pc
  }
  e.l("s_cmp_eq_u32 s95, -1");                         // were the banks converged?
  e.l("s_cselect_b32 s69, 1, 0");
  e.l("s_andn2_b64 vcc, s[96:97], s[74:75]");          // the lanes left waiting
  e.l("s_cbranch_vccz %s_conv", p.c_str());
  wave_min_vpc(e, "vcc", "s63");
  e.l("s_lshl_b32 s63, s63, 5");
  e.l("s_mov_b32 s95, s63");
  // (s69 = 1 when the banks were the converged ones)
  e.l("s_cmp_eq_u32 s69, 0");
  e.l("s_cbranch_scc1 %s_disp", p.c_str());
  e.l("s_add_u32 s70, s70, 0x%x", 2u * TC_BANK_BYTES);  // C -> D banks
  e.l("s_addc_u32 s71, s71, 0");
  e.l("s_branch %s_bankb", p.c_str());
  e.l("%s_conv:", p.c_str());
  e.l("s_mov_b32 s63, -1");
  e.l("s_mov_b32 s95, -1");
  e.l("s_cmp_eq_u32 s69, 1");
  e.l("s_cbranch_scc1 %s_disp", p.c_str());
  e.l("s_sub_u32 s70, s70, 0x%x", 2u * TC_BANK_BYTES);  // D -> C banks
  e.l("s_subb_u32 s71, s71, 0");
  e.l("%s_bankb:", p.c_str());
  e.l("s_add_u32 s72, s70, 0x%x", TC_BANK_BYTES);
  e.l("s_addc_u32 s73, s71, 0");
  // (entered with the group in s[74:75], s62 = its pc, its TInstr loading, the banks of
  // the right mode; split paths jump here directly)
  e.l("%s_disp:", p.c_str());
  e.l("s_mov_b64 exec, s[74:75]");
  e.l("s_cmp_eq_u32 s64, 0");                          // budget spent: to the kernel
  e.l("s_cbranch_scc1 %s_out", p.c_str());
  e.l("s_waitcnt lgkmcnt(0)");
  e.l("s_add_u32 s68, s70, s76");
  e.l("s_addc_u32 s69, s71, 0");
  e.l("s_setpc_b64 s[68:69]");
  e.l("%s_out:", p.c_str());
  e.l("s_add_u32 s68, s70, %u", TC_JIT_XS);
  e.l("s_addc_u32 s69, s71, 0");
  e.l("s_setpc_b64 s[68:69]");
}

// Lmerge (the group reached OTHER or the count limit: its pc is PCOFF) and Lsched.
// hybrid (trip mode beside SIMT scheduling, jit_source): a wave whose lanes are not all at
// one pc goes to the trips (Ltin) instead of picking a group; the trips come back here
// once every lane is at one pc again.
std::string simt_sched(bool hybrid, bool depth) {
  Em e;
  e.l(".p2align 6");
  e.l("Lmerge:");
  e.l("v_lshrrev_b32_e64 %s, 5, s62", VPC);
  flush(e);
  e.l("Lsched:");
  if (hybrid) {
    e.l("s_mov_b64 exec, s[96:97]");
    e.l("s_nop 4");
    e.l("v_readfirstlane_b32 s68, %s", VPC);
    e.l("s_nop 1");
    e.l("v_cmp_ne_u32_e64 vcc, s68, %s", VPC);
    e.l("s_cbranch_vccz Lsc_one");
    e.l("s_waitcnt lgkmcnt(0)");   // (a TInstr prefetch must land: the trips use s[76:81])
    long_jump(e, "Ltin", "Lsc_tq");
    e.l("Lsc_one:");
  }
  sched_block(e, "Lsc", nullptr, depth);
  return e.o;
}

// ---------------------------------------------------------------- scan loops
// A run that IS a load-scan loop (Hoare partition's `while (a[i] < p) i++`): exactly
//   x += d (I32_ADD_I / I32_SUB_I in place, d a multiple of 4, |d| <= 64)
//   y = i32.load(x + off)
//   br_<cmp> y, p (or p, y; p loop-invariant; an immediate form) back to the run's start
// runs kTripScan iterations per trip in trip mode (trip_scan_stage): every lane's next
// loads go out together, then each lane's exit iteration is found in order.
constexpr uint32_t kTripScan = 4;   // trip mode: scan iterations per trip (trip_scan_stage)
constexpr uint32_t kTripBatch = 4;  // trip mode: lane-test compares issued together (trip_source)
constexpr uint32_t kTripGuard = 4;  // trip mode: a function's runs share one range test from this many
// (mem: the memory the load reads -- 0, or k >= 1 for an XLD of a 32-bit word, whose
// window is checked against minp, memory k's declared minimum: emit_xmem)
struct ScanLoop { uint32_t x, y, off; int32_t d; bool y_first; uint32_t mem = 0, minp = 0; };

bool scan_loop_of(const Program &P, const JitRun &r, ScanLoop *sl) {
  if (r.len != 3) return false;
  const DInstr &i0 = P.code[r.pc], &i1 = P.code[r.pc + 1], &i2 = P.code[r.pc + 2];
  const uint16_t o0 = op_of(i0), o1 = op_of(i1), o2 = op_of(i2);
  if ((o0 != OP_I32_ADD_I && o0 != OP_I32_SUB_I) || (i0.w1 & 0xFFFFu) != (i0.w2 & 0xFFFFu)) return false;
  if (i0.w3 == 0 || i0.w3 % 4 || i0.w3 > 64) return false;
  const uint32_t x = i0.w1 & 0xFFFFu;
  const bool xl = o1 == OP_XLD && xmop(i1) == OP_LD32;   // (memory k >= 1: k in the b field)
  if ((o1 != OP_LD32 && !xl) || (i1.w1 & 0xFFFFu) != x || (i1.w2 & 0xFFFFu) == x) return false;
  if (xl && ((i1.w1 >> 16) == 0 || (i1.w1 >> 16) > P.xmems.size())) return false;
  const uint32_t y = i1.w2 & 0xFFFFu;
  if (!is_branch_op(o2) || o2 == OP_JMP || o2 == OP_BR_IF || o2 == OP_BR_UNLESS || i2.w3 != r.pc) return false;
  const uint32_t a = i2.w1 & 0xFFFFu, b = i2.w1 >> 16;
  bool y_first;
  if (o2 >= OP_BR_EQ_I) {
    if (a != y) return false;
    y_first = true;
  } else if (a == y && b != y && b != x) {
    y_first = true;
  } else if (b == y && a != y && a != x) {
    y_first = false;
  } else {
    return false;
  }
  if (uint64_t(i1.w3) + 64u * 2 * kTripScan + 4 > 0xFFFFFFFFull) return false;   // (the window, with room)
  *sl = ScanLoop{x, y, i1.w3, o0 == OP_I32_ADD_I ? int32_t(i0.w3) : -int32_t(i0.w3), y_first};
  if (xl) {
    sl->mem = i1.w1 >> 16;
    sl->minp = P.xmems[sl->mem - 1].min;
  }
  return true;
}

// the scan loop's branch condition (true = go round) with the loaded value in `val`
void scan_cond(Em &e, const DInstr &I, const ScanLoop &sl, const char *val) {
  const uint16_t op = op_of(I);
  const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16;
  if (op >= OP_BR_EQ_I) {
    const uint16_t k = uint16_t(op - OP_BR_EQ_I);
    e.l("v_cmp_%s32_e32 vcc, %d, %s", cmp_kind(cmp_swap(k)), int32_t(int16_t(b)), val);
  } else {
    const uint16_t k = uint16_t(op - OP_BR_EQ);
    if (sl.y_first) e.l("v_cmp_%s32_e32 vcc, %s, %s", cmp_kind(cmp_swap(k)), e.v(b), val);   // p CMP' y
    else e.l("v_cmp_%s32_e32 vcc, %s, %s", cmp_kind(k), e.v(a), val);                        // p CMP y
  }
}


// the cells an instruction writes, exactly for the 32-bit results (written() counts c + 1
// too; true), else as written() (false)
bool written_exact(const DInstr &I, std::vector<uint32_t> *out) {
  const uint32_t c = I.w2 & 0xFFFFu;
  switch (op_of(I)) {
    case OP_I32_ADD: case OP_I32_ADD3: case OP_I32_ADD_I: case OP_I32_AND: case OP_I32_AND_I:
    case OP_I32_CLZ: case OP_I32_CTZ: case OP_I32_EQ: case OP_I32_EQZ: case OP_I32_EQ_I:
    case OP_I32_EXT16S: case OP_I32_EXT8S: case OP_I32_GE_S: case OP_I32_GE_S_I:
    case OP_I32_GE_U: case OP_I32_GE_U_I: case OP_I32_GT_S: case OP_I32_GT_S_I:
    case OP_I32_GT_U: case OP_I32_GT_U_I: case OP_I32_LE_S: case OP_I32_LE_S_I:
    case OP_I32_LE_U: case OP_I32_LE_U_I: case OP_I32_LT_S: case OP_I32_LT_S_I:
    case OP_I32_LT_U: case OP_I32_LT_U_I: case OP_I32_MUL: case OP_I32_MUL_I: case OP_I32_NE:
    case OP_I32_NE_I: case OP_I32_OR: case OP_I32_OR_I: case OP_I32_POPCNT: case OP_I32_ROTL:
    case OP_I32_ROTL_I: case OP_I32_ROTR: case OP_I32_ROTR_I: case OP_I32_SHL:
    case OP_I32_SHL_I: case OP_I32_SHR_S: case OP_I32_SHR_S_I: case OP_I32_SHR_U:
    case OP_I32_SHR_U_I: case OP_I32_SUB: case OP_I32_SUB_I: case OP_I32_XOR:
    case OP_I32_XOR_I: case OP_I32_XOR_ROTL_I: case OP_I32_XOR_ROTR_I: case OP_CONST32:
    case OP_MOV32: case OP_LD32: case OP_LD8S32: case OP_LD8U32: case OP_LD16S32:
    case OP_LD16U32:
      out->assign(1, c);
      return true;
    case OP_I32_ADD_XROTR_I: *out = {c, I.w2 >> 16}; return true;
    case OP_I32_ADD3_XROTR_I: *out = {c, I.w3 & 0xFFFFu}; return true;
    default: written(I, out); return false;
  }
}

// ---------------------------------------------------------------- NaN payload liveness
// The compiled runs give every NaN result of an f32/f64 add/sub/mul the payload the
// reference's x86 build produces (Em::nan_fix: a compare and a branch per result). That
// only matters where the payload can be observed: stored, returned, kept in a global,
// passed to a call, or read as bits by an op whose result can be. A float compare sees
// every NaN alike. nan_observable() is a backward dataflow over the program's cells:
// obs(pc) = the cells whose bits may still reach such a sink after instruction pc; an
// add/sub/mul whose result is in no obs(pc) needs no fix (C5: the Mandelbrot iteration's
// z values only ever reach a compare). Unmodelled instructions make everything they name
// observable and kill nothing; calls, host calls and tail calls make every cell
// observable; globals always are (the host reads them after a trap or an interrupt).
// Returns per pc: 1 = the instruction's result may be observed.
// live (non-null): plain liveness instead -- every source of a result is live when the
// instruction runs (float compares and truncations included, their operands taken 4 cells
// wide), and *live receives the cells live before each pc (bit sets of total_cells() + 8)
std::vector<uint8_t> nan_observable(const Program &P, std::vector<std::vector<uint64_t>> *live = nullptr) {
  const size_t n = P.code.size();
  const uint32_t nc = P.total_cells() + 8;   // (+8: 4-wide over-approximations stay in range)
  const size_t W = (nc + 63) / 64;
  typedef std::vector<uint64_t> Set;
  std::vector<Set> before(n + 1, Set(W, 0));
  auto put = [&](Set &s, uint32_t c, uint32_t k) {
    for (uint32_t q = 0; q < k; q++)
      if (c + q < nc) s[(c + q) >> 6] |= 1ull << ((c + q) & 63);
  };
  auto kill = [&](Set &s, uint32_t c, uint32_t k) {
    for (uint32_t q = 0; q < k; q++)
      if (c + q < nc) s[(c + q) >> 6] &= ~(1ull << ((c + q) & 63));
  };
  auto any = [&](const Set &s, uint32_t c, uint32_t k) {
    for (uint32_t q = 0; q < k; q++)
      if (c + q < nc && (s[(c + q) >> 6] >> ((c + q) & 63) & 1)) return true;
    return false;
  };
  Set all(W, ~0ull), globals(W, 0);
  put(globals, 0, P.global_cells);
  std::vector<uint8_t> res(n, 1);
  for (bool changed = true; changed;) {
    changed = false;
    for (size_t pc = n; pc-- > 0;) {
      const DInstr &I = P.code[pc];
      const uint16_t op = op_of(I);
      const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16, c = I.w2 & 0xFFFFu, d = I.w2 >> 16;
      Set after = globals, s;
      auto succ = [&](size_t t) {
        if (t <= n) for (size_t w = 0; w < W; w++) after[w] |= before[t][w];
      };
      // what the instruction does with cells: prop = its results carry its sources' bits
      // (sources observable when a result is), hide = a float compare, sink = every cell it
      // names is observable
      uint32_t src[3][2] = {{0, 0}, {0, 0}, {0, 0}}, dst[2] = {0, 0};   // (cell, count)
      enum { PROP, HIDE, SINK, ALL, EXIT } kind = SINK;
      auto bin = [&](uint32_t w, uint32_t rw) { src[0][0] = a; src[0][1] = w; src[1][0] = b; src[1][1] = w; dst[0] = c; dst[1] = rw; };
      auto un = [&](uint32_t w, uint32_t rw) { src[0][0] = a; src[0][1] = w; dst[0] = c; dst[1] = rw; };
      std::vector<uint32_t> wx;
      switch (op) {
        case OP_F32_ADD: case OP_F32_SUB: case OP_F32_MUL: case OP_F32_DIV: case OP_F32_MIN:
        case OP_F32_MAX: case OP_F32_COPYSIGN: kind = PROP; bin(1, 1); break;
        case OP_F64_ADD: case OP_F64_SUB: case OP_F64_MUL: case OP_F64_DIV: case OP_F64_MIN:
        case OP_F64_MAX: case OP_F64_COPYSIGN: kind = PROP; bin(2, 2); break;
        case OP_F32_ABS: case OP_F32_NEG: case OP_F32_CEIL: case OP_F32_FLOOR: case OP_F32_TRUNC:
        case OP_F32_NEAREST: case OP_F32_SQRT: case OP_MOV32: kind = PROP; un(1, 1); break;
        case OP_F64_ABS: case OP_F64_NEG: case OP_F64_CEIL: case OP_F64_FLOOR: case OP_F64_TRUNC:
        case OP_F64_NEAREST: case OP_F64_SQRT: case OP_MOV64: kind = PROP; un(2, 2); break;
        case OP_F32_DEMOTE_F64: kind = PROP; un(2, 1); break;
        case OP_F64_PROMOTE_F32: kind = PROP; un(1, 2); break;
        case OP_MOV128: case OP_V_NOT: case OP_V_F32X4_ABS: case OP_V_F32X4_NEG: case OP_V_F32X4_SQRT:
        case OP_V_F64X2_ABS: case OP_V_F64X2_NEG: case OP_V_F64X2_SQRT: kind = PROP; un(4, 4); break;
        case OP_CONST32: kind = PROP; dst[0] = c; dst[1] = 1; break;
        case OP_CONST64: kind = PROP; dst[0] = c; dst[1] = 2; break;
        case OP_CONST128: kind = PROP; dst[0] = c; dst[1] = 4; break;
        case OP_V_I32X4_SPLAT: case OP_V_F32X4_SPLAT: kind = PROP; un(1, 4); break;
        case OP_V_I64X2_SPLAT: case OP_V_F64X2_SPLAT: kind = PROP; un(2, 4); break;
        case OP_V_AND: case OP_V_OR: case OP_V_XOR: case OP_V_ANDNOT: case OP_V_I32X4_ADD:
        case OP_V_I32X4_SUB: case OP_V_I32X4_MUL: case OP_V_I64X2_ADD: case OP_V_I64X2_SUB:
        case OP_V_F32X4_ADD: case OP_V_F32X4_SUB: case OP_V_F32X4_MUL: case OP_V_F32X4_DIV:
        case OP_V_F32X4_MIN: case OP_V_F32X4_MAX: case OP_V_F32X4_PMIN: case OP_V_F32X4_PMAX:
        case OP_V_F64X2_ADD: case OP_V_F64X2_SUB: case OP_V_F64X2_MUL: case OP_V_F64X2_DIV:
        case OP_V_F64X2_MIN: case OP_V_F64X2_MAX: case OP_V_F64X2_PMIN: case OP_V_F64X2_PMAX:
          kind = PROP; bin(4, 4); break;
        case OP_V_EXTRACT32: kind = PROP; un(4, 1); break;
        case OP_V_EXTRACT64: kind = PROP; un(4, 2); break;
        case OP_V_REPLACE32: kind = PROP; bin(4, 4); src[1][1] = 1; break;
        case OP_V_REPLACE64: kind = PROP; bin(4, 4); src[1][1] = 2; break;
        case OP_V_ANY_TRUE: kind = PROP; un(4, 1); break;
        case OP_F32_EQ: case OP_F32_NE: case OP_F32_LT: case OP_F32_GT: case OP_F32_LE: case OP_F32_GE:
          kind = HIDE; dst[0] = c; dst[1] = 1; break;
        case OP_F64_EQ: case OP_F64_NE: case OP_F64_LT: case OP_F64_GT: case OP_F64_LE: case OP_F64_GE:
          kind = HIDE; dst[0] = c; dst[1] = 1; break;
        case OP_V_F32X4_EQ: case OP_V_F32X4_NE: case OP_V_F32X4_LT: case OP_V_F32X4_GT:
        case OP_V_F32X4_LE: case OP_V_F32X4_GE: case OP_V_F64X2_EQ: case OP_V_F64X2_NE:
        case OP_V_F64X2_LT: case OP_V_F64X2_GT: case OP_V_F64X2_LE: case OP_V_F64X2_GE:
          kind = HIDE; dst[0] = c; dst[1] = 4; break;
        case OP_I64_ADD: case OP_I64_SUB: case OP_I64_MUL: case OP_I64_AND: case OP_I64_OR:
        case OP_I64_XOR: case OP_I64_SHL: case OP_I64_SHR_S: case OP_I64_SHR_U: case OP_I64_ROTL:
        case OP_I64_ROTR: kind = PROP; bin(2, 2); break;
        case OP_I64_EQ: case OP_I64_NE: case OP_I64_LT_S: case OP_I64_LT_U: case OP_I64_GT_S:
        case OP_I64_GT_U: case OP_I64_LE_S: case OP_I64_LE_U: case OP_I64_GE_S: case OP_I64_GE_U:
          kind = PROP; bin(2, 1); break;
        case OP_I64_ADD_I: case OP_I64_SUB_I: case OP_I64_MUL_I: case OP_I64_AND_I: case OP_I64_OR_I:
        case OP_I64_XOR_I: case OP_I64_SHL_I: case OP_I64_SHR_S_I: case OP_I64_SHR_U_I:
        case OP_I64_ROTL_I: case OP_I64_ROTR_I: case OP_I64_CLZ: case OP_I64_CTZ: case OP_I64_POPCNT:
        case OP_I64_EXT8S: case OP_I64_EXT16S: case OP_I64_EXT32S: kind = PROP; un(2, 2); break;
        case OP_I64_EQ_I: case OP_I64_NE_I: case OP_I64_LT_S_I: case OP_I64_LT_U_I: case OP_I64_GT_S_I:
        case OP_I64_GT_U_I: case OP_I64_LE_S_I: case OP_I64_LE_U_I: case OP_I64_GE_S_I:
        case OP_I64_GE_U_I: case OP_I64_EQZ: kind = PROP; un(2, 1); break;
        case OP_I64_EXTEND_I32_S: case OP_I64_EXTEND_I32_U: case OP_F64_CONVERT_I32_S:
        case OP_F64_CONVERT_I32_U: kind = PROP; un(1, 2); break;
        case OP_F32_CONVERT_I32_S: case OP_F32_CONVERT_I32_U: kind = PROP; un(1, 1); break;
        case OP_F32_CONVERT_I64_S: case OP_F32_CONVERT_I64_U: kind = PROP; un(2, 1); break;
        case OP_F64_CONVERT_I64_S: case OP_F64_CONVERT_I64_U: kind = PROP; un(2, 2); break;
        case OP_SELECT32: case OP_SELECT64: case OP_SELECT128: {
          const uint32_t w = op == OP_SELECT32 ? 1 : op == OP_SELECT64 ? 2 : 4;
          kind = PROP; bin(w, w); src[2][0] = d; src[2][1] = 1; break;
        }
        case OP_V_I8X16_EQ: case OP_V_I8X16_NE: case OP_V_I16X8_EQ: case OP_V_I16X8_NE:
        case OP_V_I32X4_EQ: case OP_V_I32X4_NE: case OP_V_I32X4_LT_S: case OP_V_I32X4_LT_U:
        case OP_V_I32X4_GT_S: case OP_V_I32X4_GT_U: case OP_V_I32X4_LE_S: case OP_V_I32X4_LE_U:
        case OP_V_I32X4_GE_S: case OP_V_I32X4_GE_U: case OP_V_I64X2_EQ: case OP_V_I64X2_NE:
        case OP_V_I64X2_LT_S: case OP_V_I64X2_GT_S: case OP_V_I64X2_LE_S: case OP_V_I64X2_GE_S:
        case OP_V_I64X2_MUL: case OP_V_I8X16_ADD: case OP_V_I8X16_SUB: case OP_V_I16X8_ADD:
        case OP_V_I16X8_SUB: case OP_V_I16X8_MUL: kind = PROP; bin(4, 4); break;
        case OP_V_I8X16_BITMASK: case OP_V_I16X8_BITMASK: case OP_V_I32X4_BITMASK:
        case OP_V_I64X2_BITMASK: case OP_V_I8X16_ALL_TRUE: case OP_V_I16X8_ALL_TRUE:
        case OP_V_I32X4_ALL_TRUE: case OP_V_I64X2_ALL_TRUE: kind = PROP; un(4, 1); break;
        // float -> int: a NaN traps or saturates whatever its payload
        case OP_I32_TRUNC_F32_S: case OP_I32_TRUNC_F32_U: case OP_I32_TRUNC_F64_S:
        case OP_I32_TRUNC_F64_U: case OP_I32_TRUNC_SAT_F32_S: case OP_I32_TRUNC_SAT_F32_U:
        case OP_I32_TRUNC_SAT_F64_S: case OP_I32_TRUNC_SAT_F64_U:
          kind = HIDE; dst[0] = c; dst[1] = 1; break;
        case OP_I64_TRUNC_F32_S: case OP_I64_TRUNC_F32_U: case OP_I64_TRUNC_F64_S:
        case OP_I64_TRUNC_F64_U: case OP_I64_TRUNC_SAT_F32_S: case OP_I64_TRUNC_SAT_F32_U:
        case OP_I64_TRUNC_SAT_F64_S: case OP_I64_TRUNC_SAT_F64_U:
          kind = HIDE; dst[0] = c; dst[1] = 2; break;
        case OP_NOP_CNT: kind = PROP; break;
        case OP_ZERO_LOCALS: kind = PROP; dst[0] = a; dst[1] = b; break;
        case OP_RET: case OP_UNREACHABLE: kind = EXIT; break;
        case OP_CALL: case OP_CALL_INDIRECT: case OP_HOST_CALL: case OP_TAIL_CALL:
        case OP_TAIL_CALL_INDIRECT: kind = ALL; break;
        default:
          // exact single-result 32-bit integer ops (not the loads: their address can trap)
          if (!mem_bytes(op) && written_exact(I, &wx) && wx.size() == 1 && wx[0] == c) {
            kind = PROP;
            src[0][0] = a; src[0][1] = 1; src[1][0] = b; src[1][1] = 1; dst[0] = c; dst[1] = 1;
            src[2][0] = d; src[2][1] = 1;   // (I32_ADD3's third operand)
          }
          // (the other DBC_CTL ops may trap -- an exit, after which only globals and
          // memory remain -- or leave the core; their successor is still pc + 1)
          break;
      }
      // successors
      if (kind == ALL) {
        s = all;
      } else if (kind == EXIT) {
        s = globals;
        if (op == OP_RET) put(s, a, b);
      } else {
        if (op == OP_BR_TABLE) {
          for (uint32_t k = 0; k <= b; k++)
            if (2 * (size_t(I.w3) + k) < P.brtab.size()) succ(P.brtab[2 * (size_t(I.w3) + k)]);
        } else {
          if (op != OP_JMP) succ(pc + 1);
          if (is_branch_op(op) || op == OP_BR_IF_MOV1 || op == OP_BR_IF_MOV2) succ(I.w3);
        }
        s = after;
        if (kind == PROP || kind == HIDE) {
          const bool used = any(after, dst[0], dst[1]);
          if (dst[1]) res[pc] = used ? 1 : 0;
          kill(s, dst[0], dst[1]);
          if (kind == PROP && (used || live))
            for (auto &x : src) put(s, x[0], x[1]);
          if (kind == HIDE && live) { put(s, a, 4); put(s, b, 4); }
        } else if (is_store_op(op)) {   // the address and the stored bits
          put(s, a, 1);
          put(s, b, std::max(1u, mem_bytes(op) / 4));
        } else if (mem_bytes(op)) {     // a load: its address; its result is memory's
          const bool w64 = op == OP_LD8S64 || op == OP_LD8U64 || op == OP_LD16S64 ||
                           op == OP_LD16U64 || op == OP_LD32S64 || op == OP_LD32U64 || op == OP_LD64;
          kill(s, c, op == OP_LD128 ? 4 : w64 ? 2 : 1);
          put(s, a, 1);
        } else if (is_branch_op(op) || op == OP_BR_TABLE) {   // i32 operands
          if (op != OP_JMP) put(s, a, 1);
          if (op >= OP_BR_EQ && op <= OP_BR_GE_U) put(s, b, 1);
        } else if (op == OP_BR_IF_MOV1 || op == OP_BR_IF_MOV2) {   // a: condition, b -> c
          put(s, a, 1);
          put(s, b, op == OP_BR_IF_MOV1 ? 1 : 2);
        } else {   // sink: every field it names, 4 wide, is observable
          put(s, a, 4); put(s, b, 4); put(s, c, 4); put(s, d, 4);
          if (op == OP_I32_ADD3_XROTR_I) put(s, I.w3 & 0xFFFFu, 1);
        }
        for (size_t w = 0; w < W; w++) s[w] |= globals[w];
      }
      if (s != before[pc]) {
        before[pc] = s;
        changed = true;
      }
    }
  }
  if (live) *live = before;
  // (debugging aid: WB_NANOBS_LIST=<file> writes per pc the flag and the cells observable
  // before it)
  if (const char *lst = getenv("WB_NANOBS_LIST"))
    if (FILE *f = fopen(lst, "w")) {
      for (size_t pc = 0; pc < n; pc++) {
        fprintf(f, "%4zu %d", pc, int(res[pc]));
        for (uint32_t x = 0; x < nc; x++)
          if (before[pc][x >> 6] >> (x & 63) & 1) fprintf(f, " %u", x);
        fprintf(f, "\n");
      }
      fclose(f);
    }
  return res;
}

// Loop-carried memory forwarding. A loop whose body is a run R ending in an inlined leaf
// call and the post-call run Pp branching back to R's start (C2: the chain loop around
// BLAKE3's compression) reads the words its previous trip stored or loaded: the callee's
// 32-bit accesses all go to constant addresses (i32.const arguments, params never
// written) and nothing else on the loop touches memory. Every access then also keeps its
// word in a VGPR above every cell (F); the inlined call's end goes on in a copy of Pp
// (suffix p) whose taken branch enters a copy of R (suffix c) where the callee's loads
// are moves from F: no loads, hence no waits behind the previous trip's stores (vmcnt
// retires in issue order). Stores stay real (memory is always current) and a copy's
// lanes are the group that ran the trip before (the fast path keeps exec), so every
// lane's F words are its own memory's. The c copy skips the load-only groups' checks:
// the first trip, in R, checked the same constant addresses and memory never shrinks.
struct FwdPlan {
  size_t post = 0;                                       // Pp (run index)
  std::vector<int64_t> addr;                             // callee body index -> address
  std::map<uint32_t, uint32_t> freg;                     // address -> VGPR
  std::vector<std::pair<uint32_t, uint32_t>> end_copy;   // (VGPR, physical cell)
  std::vector<uint8_t> copy_now;   // body index: a load whose cell changes later (copy at once)
};

bool fwd_plan(const Program &P, const std::vector<JitRun> &runs, size_t k, size_t f, size_t post,
              FwdPlan *out) {
  const JitRun &R = runs[k], &F = runs[f], &Q = runs[post];
  const DInstr &call = P.code[R.pc + R.len - 1], &br = P.code[Q.pc + Q.len - 1];
  if (!is_branch_op(op_of(br)) || br.w3 != R.pc) return false;
  const uint32_t fb = P.global_cells, L = call.w1 & 0xFFFFu, off = L - fb;
  for (uint32_t i = 0; i < Q.len; i++)
    if (mem_bytes(op_of(P.code[Q.pc + i]))) return false;
  std::map<uint32_t, uint32_t> cst;   // physical cell -> constant
  std::vector<uint32_t> wr;
  auto step = [&](const DInstr &I, uint32_t sh) {
    const uint16_t op = op_of(I);
    const uint32_t a = I.w1 & 0xFFFFu, c = I.w2 & 0xFFFFu;
    auto ph = [&](uint32_t x) { return x >= fb ? x + sh : x; };
    if (op == OP_CONST32) { cst[ph(c)] = I.w3; return; }
    if (op == OP_MOV32 && cst.count(ph(a))) { cst[ph(c)] = cst[ph(a)]; return; }
    written_exact(I, &wr);
    for (uint32_t x : wr) cst.erase(ph(x));
  };
  for (uint32_t i = 0; i + 1 < R.len; i++) {
    if (mem_bytes(op_of(P.code[R.pc + i]))) return false;
    step(P.code[R.pc + i], 0);
  }
  const uint32_t nloc = call.w2 & 0xFFFFu, nargs = call.w1 >> 16;
  for (uint32_t q = 0; q < nloc; q++) cst.erase(L + nargs + q);   // (the callee's zeroed locals)
  out->post = post;
  out->addr.assign(F.len, -1);
  out->copy_now.assign(F.len, 0);
  std::map<uint32_t, std::pair<bool, uint32_t>> lastacc;   // address -> (load, body index)
  for (uint32_t i = 0; i + 1 < F.len; i++) {
    const DInstr &I = P.code[F.pc + i];
    const uint16_t op = op_of(I);
    if (mem_bytes(op)) {
      const uint32_t a = I.w1 & 0xFFFFu, pa = a >= fb ? a + off : a;
      if ((op != OP_LD32 && op != OP_ST32) || !cst.count(pa)) return false;
      const uint64_t A = uint64_t(cst[pa]) + I.w3;
      if ((A & 3) || A + 4 > 0xFFFFFFFFull) return false;
      out->addr[i] = int64_t(A);
      lastacc[uint32_t(A)] = {op == OP_LD32, i};
    }
    step(I, off);
  }
  uint32_t prev = 0;
  bool first = true;
  for (auto &kv : lastacc) {   // (ordered) distinct words must not overlap
    if (!first && kv.first - prev < 4) return false;
    prev = kv.first;
    first = false;
  }
  const uint32_t base = uint32_t(P.total_cells()) + off;
  if (lastacc.empty() || lastacc.size() > 64 || base + lastacc.size() > TC_VF_CELLS) return false;
  uint32_t n = 0;
  for (auto &kv : lastacc) {
    const uint32_t v = 128 + base + n++;
    out->freg[kv.first] = v;
    if (!kv.second.first) continue;
    // a word last loaded: copied at the callee's end if its cell still holds it then,
    // else right after the load
    const DInstr &ld = P.code[F.pc + kv.second.second];
    const uint32_t c = ld.w2 & 0xFFFFu;
    bool kept = true;
    for (uint32_t i = kv.second.second + 1; kept && i + 1 < F.len; i++) {
      written_exact(P.code[F.pc + i], &wr);
      kept = std::find(wr.begin(), wr.end(), c) == wr.end();
    }
    if (kept) out->end_copy.push_back({v, c >= fb ? c + off : c});
    else out->copy_now[kv.second.second] = 1;
  }
  return true;
}

// ---------------------------------------------------------------- trip mode
// SIMT scheduling runs one group of lanes at a time -- the lanes at the lowest pc -- and a
// group waits out the latency of each load it makes. Where lanes part ways on loaded data
// (C3's Hoare scans: every lane leaves its `while (a[i] < p) i++` after its own number of
// steps) the groups are small (4.0 active lanes per VALU instruction, 62% of wave cycles
// waiting on memory: profiles/r03b_c3_counters.md), so the wave pays one memory latency
// per few lane-steps. Trip mode runs every lane instead: in one trip each lane of the wave
// that waits at the start of a compiled run executes that whole run, whichever it is,
// and all the runs' loads are in flight together:
//   stage A  for each run with lanes: EXEC = its lanes, its instructions up to its loads
//            and the loads themselves (nothing here reads a loaded cell: trip_split);
//   one s_waitcnt vmcnt(0) for every load of the trip;
//   stage B  for each run with lanes: the rest of the run and its transfer, per lane
//            (VPC = the lane's next pc, VCNT += what it retired, the taken count
//            corrections per lane; calls, returns and br_table per lane too).
// The lanes' register state is their own (VGPRs under disjoint EXEC masks), so a run's
// temporaries survive from its stage A to its stage B. TPC (v98) = the pc a lane started
// the trip at: a lane moved to another run in stage B runs that one in the next trip.
// Lanes at a pc where no run starts wait outside the trips (OUTSIDE s[76:77]), and so do
// lanes that must leave before an instruction (a failed bounds/alignment check, a call
// stack past its LDS part, a return from the entry function: ESC s[78:79], Em::trip_leave).
// Trips go on while more lanes are in the runs than outside them; then escapes go to the
// C++ step (xh) and the other outside lanes to the scheduler's pick among them (their
// handlers, Ltq), and they come back through a run's entry. Every trip costs 256 of the
// core's budget (or the longest run's count, if more): the core returns to the kernel
// (limits, interrupts) every 4K trips, and no lane retires more than the budget plus one run.
namespace {
const char *const TPC = "v98";

// does I name a cell of `set` in any operand field (one cell per field for the 32-bit
// ops of written_exact, else conservatively 4)
bool names_any(const DInstr &I, const std::vector<uint8_t> &set) {
  const uint32_t f[5] = {I.w1 & 0xFFFFu, I.w1 >> 16, I.w2 & 0xFFFFu, I.w2 >> 16,
                         op_of(I) == OP_I32_ADD3_XROTR_I ? (I.w3 & 0xFFFFu) : 0xFFFFu};
  std::vector<uint32_t> w;
  const uint32_t width = written_exact(I, &w) ? 1u : 4u;
  for (uint32_t x : f)
    for (uint32_t k = 0; k < width; k++)
      if (x + k < set.size() && set[x + k]) return true;
  return false;
}

// stage A of a run = its instructions before trip_split: up to its first store or
// POST_CALL past the first, or the first instruction that names a cell loaded before it;
// 0 when that prefix loads nothing (all in stage B)
uint32_t trip_split(const Program &P, const JitRun &r, uint32_t nbody) {
  std::vector<uint8_t> loaded(TC_VF_CELLS + 8, 0);
  uint32_t s = 0;
  bool any = false;
  for (uint32_t i = 0; i < nbody; i++) {
    const DInstr &I = P.code[r.pc + i];
    const uint16_t op = op_of(I);
    if (names_any(I, loaded) || (op == OP_POST_CALL && i) || is_store_op(op) || op == OP_XST) break;
    if (mem_bytes(op) || op == OP_XLD) {
      const uint32_t c = I.w2 & 0xFFFFu;
      for (uint32_t k = 0; k < load_cells(op == OP_XLD ? xmop(I) : op); k++) loaded[c + k] = 1;
      any = true;
    }
    s = i + 1;
  }
  return any ? s : 0;
}
}  // namespace

// Trip-mode scan loops (trip_source): the lanes of a scan run whose window of U
// addresses is in bounds and aligned (flag v112 = 1) load all U words in stage A
// (v108..v108+U-1) and find their exit in stage B; the others (v112 = 0) run the plain
// stage code that follows (exec = them; the stage ends at once when there are none).
// Entered with EXEC = the run's lanes in this trip. Temporaries survive from stage A to
// stage B per lane (other runs execute under disjoint EXEC masks).
// slot: the run's load-cache VGPRs {address, value} (-1: none) -- invalidated for all its
// lanes in stage A, set to (x + off, y) by the window lanes that leave the scan in stage B.
// T2 = the lanes whose scan window (bytes (x + d*j) + off .. +3 for j = 1..U) is out of
// bounds, unaligned or wraps x + d*j (as the SIMT scan block)
void scan_window_fails(Em &e, const ScanLoop &sl, uint32_t U) {
  const uint32_t up = sl.off + (sl.d > 0 ? uint32_t(sl.d) * U : 0u) + 3u;
  e.l("v_add_co_u32_e32 %s, vcc, 0x%x, %s", X0, up, e.v(sl.x));
  e.l("v_lshrrev_b32_e32 %s, 16, %s", X1, X0);
  if (sl.mem) {
    e.l("s_mov_b32 s68, 0x%x", sl.minp);
    e.l("v_cmp_le_u32_e64 %s, s68, %s", T2, X1);
  } else {
    e.l("v_cmp_ge_u32_e64 %s, %s, %s", T2, X1, PAGES);
  }
  e.l("s_or_b64 %s, %s, vcc", T2, T2);
  e.l("v_add_u32_e32 %s, 0x%x, %s", Y0, sl.off, e.v(sl.x));
  if (sl.d < 0) {
    e.l("v_cmp_gt_u32_e32 vcc, 0x%x, %s", uint32_t(-sl.d) * U, e.v(sl.x));
    e.l("s_or_b64 %s, %s, vcc", T2, T2);
  }
  e.l("v_and_b32_e32 %s, 3, %s", Y1, Y0);
  e.l("v_cmp_ne_u32_e32 vcc, 0, %s", Y1);
  e.l("s_or_b64 %s, %s, vcc", T2, T2);
}

// the scan window's U words into dst[0..U-1] (the window checked)
void scan_window_words(Em &e, const ScanLoop &sl, uint32_t U, const std::vector<std::string> &dst);
void scan_window_loads(Em &e, const ScanLoop &sl, uint32_t U, const std::vector<std::string> &dst) {
  if (sl.mem) xmem_lane_base(e, sl.mem);   // (RP: the lane's word 0 of memory k)
  // One 16-byte load per lane whose window lies in one granule (granules of 16 bytes or
  // more, |d| = 4, the destination registers consecutive in address order), the word by
  // word path for the others (WB_TRIP_X4=0: word by word always)
  const uint32_t g = sl.mem ? g_xlog : e.g;
  int r = -1;
  if (U == 4 && g >= 2 && (sl.d == 4 || sl.d == -4) && !(getenv("WB_TRIP_X4") && getenv("WB_TRIP_X4")[0] == '0')) {
    int lo = -1;
    bool ok = true;
    for (uint32_t q = 0; q < 4 && ok; q++) {   // q-th word in address order
      const std::string &reg = dst[sl.d > 0 ? q : 3 - q];
      const int v = reg.size() > 1 && reg[0] == 'v' ? atoi(reg.c_str() + 1) : -1;
      if (q == 0) lo = v;
      ok = v >= 0 && v == lo + int(q);
    }
    if (ok && !(lo & 1)) r = lo;   // (VGPR tuples start at even registers)
  }
  if (r < 0) { scan_window_words(e, sl, U, dst); return; }
  static thread_local int nx4 = 0;
  const std::string id = std::to_string(nx4++);
  const char *base = sl.mem ? RP : MEM;
  const uint32_t lo_off = uint32_t(int64_t(sl.off) + (sl.d > 0 ? 4 : -16));
  e.l("v_add_u32_e32 %s, 0x%x, %s", Y0, lo_off, e.v(sl.x));
  e.l("v_and_b32_e32 %s, 0x%x, %s", Y1, (4u << g) - 1u, Y0);
  e.l("v_cmp_ge_u32_e32 vcc, 0x%x, %s", (4u << g) - 16u, Y1);   // the window in one granule
  e.l("s_mov_b64 s[68:69], exec");
  e.l("s_and_b64 exec, exec, vcc");
  e.l("s_cbranch_execz Lx4a%s", id.c_str());
  if (!sl.mem) {
    granule_addr(e, XP, Y0, MEM);
  } else {
    e.l("v_lshrrev_b32_e32 %s, %u, %s", W0, 2 + g, Y0);
    e.l("v_lshlrev_b64 %s, %u, %s", XP, 8 + g, WP);
    e.l("v_lshl_add_u64 %s, %s, 0, %s", XP, XP, base);
    e.l("v_bfe_u32 %s, %s, 0, %u", W0, Y0, 2 + g);
    e.l("v_lshl_add_u64 %s, %s, 0, %s", XP, WP, XP);
  }
  e.l("global_load_dwordx4 v[%d:%d], %s, off", r, r + 3, XP);
  e.l("Lx4a%s:", id.c_str());
  e.l("s_andn2_b64 exec, s[68:69], vcc");
  e.l("s_cbranch_execz Lx4b%s", id.c_str());
  scan_window_words(e, sl, U, dst);
  e.l("Lx4b%s:", id.c_str());
  e.l("s_mov_b64 exec, s[68:69]");
}

// (word by word: RP already set for an extra memory)
void scan_window_words(Em &e, const ScanLoop &sl, uint32_t U, const std::vector<std::string> &dst) {
  for (uint32_t j = 1; j <= U; j++) {
    e.l("v_add_u32_e32 %s, 0x%x, %s", Y0, uint32_t(int64_t(sl.off) + int64_t(sl.d) * j), e.v(sl.x));
    if (sl.mem && !g_xlog) {   // (an extra memory in the word interleave)
      e.l("v_mov_b32 %s, %s", W0, Y0);
      e.l("v_lshlrev_b64 %s, 6, %s", XP, WP);
      e.l("v_lshl_add_u64 %s, %s, 0, %s", XP, XP, RP);
    } else if (sl.mem) {       // (an extra memory in granules of 4 << g_xlog bytes)
      e.l("v_lshrrev_b32_e32 %s, %u, %s", W0, 2 + g_xlog, Y0);
      e.l("v_lshlrev_b64 %s, %u, %s", XP, 8 + g_xlog, WP);
      e.l("v_lshl_add_u64 %s, %s, 0, %s", XP, XP, RP);
      e.l("v_bfe_u32 %s, %s, 0, %u", W0, Y0, 2 + g_xlog);
      e.l("v_lshl_add_u64 %s, %s, 0, %s", XP, WP, XP);
    } else if (e.g == 0) {
      e.l("v_mov_b32 %s, %s", W0, Y0);
      e.l("v_lshlrev_b64 %s, 6, %s", XP, WP);
      e.l("v_lshl_add_u64 %s, %s, 0, %s", XP, XP, MEM);
    } else {
      granule_addr(e, XP, Y0, MEM);
    }
    e.l("global_load_dword %s, %s, off", dst[j - 1].c_str(), XP);
  }
}

// The successor-window prefetch (trip_source): in stage A of a scan run that falls into
// another scan run (Hoare's i-scan into its j-scan), every lane also loads the successor's
// window at the successor's current x into pf.v[0..U-1] and records that x in pf.x (-1:
// none). The lanes that leave the first scan in this trip then run the successor's stage B
// in the same trip (LtS) when their x still equals pf.x -- the words are still the
// memory's: pf.x is invalidated by every store of the lane and at the trips' entry.
struct ScanPrefetch { uint32_t x = 0; std::vector<std::string> v; };

void trip_scan_prefetch(Em &e, const ScanLoop &succ, uint32_t U, const ScanPrefetch &pf,
                        const std::string &L) {
  e.l("v_mov_b32 v%u, -1", pf.x);
  scan_window_fails(e, succ, U);
  e.l("s_and_b64 s[84:85], exec, %s", T2);     // (no prefetch)
  e.l("s_andn2_b64 exec, exec, %s", T2);
  e.l("s_cbranch_execz %s_pf", L.c_str());
  e.l("v_mov_b32 v%u, %s", pf.x, e.v(succ.x));
  scan_window_loads(e, succ, U, pf.v);
  e.l("%s_pf:", L.c_str());
  e.l("s_or_b64 exec, exec, s[84:85]");
}

// the window's j-th word's register (v108..v111, in address order: one 16-byte load fills
// them, scan_window_loads)
const char *scan_T(const ScanLoop &sl, uint32_t j) {
  static const char *const up[kTripScan] = {"v108", "v109", "v110", "v111"};
  static const char *const down[kTripScan] = {"v111", "v110", "v109", "v108"};
  return sl.d > 0 ? up[j] : down[j];
}

// win: (stage B, branch-free form) the window's registers when every lane of the stage has
// its window there already (LtS: the successor prefetch's), else v108.. and the v112 flag
bool scan_bf_on() { return !(getenv("WB_TRIP_SCANBF") && getenv("WB_TRIP_SCANBF")[0] == '0'); }

void trip_scan_stage(Em &e, const Program &P, const JitRun &r, const ScanLoop &sl, uint32_t U,
                     int st, bool fall_in, const std::string &L, std::pair<int, int> slot,
                     const std::vector<std::string> *win = nullptr) {
  const char *T[kTripScan];
  for (uint32_t j = 0; j < kTripScan; j++) T[j] = win && j < win->size() ? (*win)[j].c_str() : scan_T(sl, j);
  const uint32_t x = sl.x, y = sl.y, fall = r.pc + 3;
  const DInstr &br = P.code[r.pc + 2];
  const int32_t tcnt = int32_t(int16_t(br.w2 >> 16));
  if (st == 0 && slot.first >= 0) e.l("v_mov_b32 v%d, -1", slot.first);
  if (st == 0) {
    scan_window_fails(e, sl, U);
    e.l("s_and_b64 s[84:85], exec, %s", T2);     // plain lanes
    e.l("s_andn2_b64 exec, exec, %s", T2);       // window lanes
    e.l("s_cbranch_execz %s_sp", L.c_str());
    e.l("v_mov_b32 v112, 1");
    scan_window_loads(e, sl, U, std::vector<std::string>(T, T + U));
    e.l("%s_sp:", L.c_str());
    e.l("s_mov_b64 exec, s[84:85]");
    e.l("s_cbranch_execz %s", e.stage_end.c_str());
    e.l("v_mov_b32 v112, 0");
    return;
  }
  // stage B: the window lanes' exits in iteration order (s[82:83] = still looping)
  if (win) {
    e.l("s_mov_b64 s[84:85], 0");                // (every lane has its window)
  } else {
    e.l("v_cmp_ne_u32_e32 vcc, 0, v112");
    e.l("s_andn2_b64 s[84:85], exec, vcc");        // plain lanes
    e.l("s_and_b64 exec, exec, vcc");
    e.l("s_cbranch_execz %s_sb", L.c_str());
  }
  if (scan_bf_on()) {
    // Branch-free (WB_TRIP_SCANBF=0: the iteration-by-iteration form below): each lane's
    // exit iteration E (U + 1: none) and the word it ended on, from the last iteration to
    // the first; then x += d * min(E, U), the count min(E, U) * (cnt + tcnt) less the
    // untaken branch's tcnt for the lanes that leave, and those lanes' pc, cache slot and
    // place outside the trips -- exactly what the iterations one by one retire.
    const char *E = X0, *Yv = X1, *Em = Y0, *tmp = Y1;
    e.l("v_mov_b32 %s, %u", E, U + 1);
    e.l("v_mov_b32 %s, %s", Yv, T[U - 1]);
    for (uint32_t j = U; j >= 1; j--) {
      scan_cond(e, br, sl, T[j - 1]);   // vcc = goes round at iteration j
      e.l("v_cndmask_b32_e64 %s, %u, %s, vcc", E, j, E);
      if (j < U) e.l("v_cndmask_b32_e32 %s, %s, %s, vcc", Yv, T[j - 1], Yv);
    }
    e.l("v_min_u32_e32 %s, %u, %s", Em, U, E);
    auto k32 = [&](int32_t v, const char *sreg) -> std::string {   // an inline constant or an SGPR
      if (v >= -16 && v <= 64) return std::to_string(v);
      e.l("s_mov_b32 %s, 0x%x", sreg, uint32_t(v));
      return sreg;
    };
    const std::string dk = k32(sl.d, "s68");
    e.l("v_mad_i32_i24 %s, %s, %s, %s", e.v(x), Em, dk.c_str(), e.v(x));
    e.l("v_mov_b32 %s, %s", e.v(y), Yv);
    const std::string ck = k32(int32_t(r.cnt) + tcnt, "s69");
    e.l("v_mad_i32_i24 %s, %s, %s, %s", VCNT, Em, ck.c_str(), VCNT);
    e.l("v_cmp_lt_u32_e32 vcc, %u, %s", U, E);   // vcc = still going round
    if (tcnt) {
      if (-tcnt >= -16 && -tcnt <= 64) {
        e.l("v_cndmask_b32_e64 %s, %d, 0, vcc", tmp, -tcnt);
      } else {
        e.l("v_mov_b32 %s, 0x%x", tmp, uint32_t(-tcnt));
        e.l("v_cndmask_b32_e64 %s, %s, 0, vcc", tmp, tmp);
      }
      e.l("v_add_u32_e32 %s, %s, %s", VCNT, VCNT, tmp);
    }
    if (fall <= 64) {   // (VCC is a constant-bus read already: no literal beside it)
      e.l("v_cndmask_b32_e64 %s, %u, %s, vcc", VPC, fall, VPC);
    } else {
      e.l("v_mov_b32 %s, 0x%x", tmp, fall);
      e.l("v_cndmask_b32_e32 %s, %s, %s, vcc", VPC, tmp, VPC);
    }
    if (slot.first >= 0) {   // (the load cache: the word that ended the scan, and its address)
      e.l("v_add_u32_e32 %s, 0x%x, %s", tmp, sl.off, e.v(x));
      e.l("v_cndmask_b32_e32 v%d, %s, v%d, vcc", slot.first, tmp, slot.first);
      e.l("v_cndmask_b32_e32 v%d, %s, v%d, vcc", slot.second, Yv, slot.second);
    }
    if (!fall_in) {   // (the lanes that leave wait outside the trips)
      e.l("s_andn2_b64 s[68:69], exec, vcc");
      e.l("s_or_b64 s[76:77], s[76:77], s[68:69]");
    }
    e.l("%s_sb:", L.c_str());
    e.l("s_mov_b64 exec, s[84:85]");
    e.l("s_cbranch_execz %s", e.stage_end.c_str());
    return;
  }
  e.l("s_mov_b64 s[82:83], exec");
  for (uint32_t j = 1; j <= U; j++) {
    const std::string nx = L + "_n" + std::to_string(j);
    scan_cond(e, br, sl, T[j - 1]);
    e.l("s_andn2_b64 s[68:69], s[82:83], vcc");   // leave in iteration j
    e.l("s_and_b64 s[82:83], s[82:83], vcc");
    e.l("s_cmp_eq_u64 s[68:69], 0");
    e.l("s_cbranch_scc1 %s", nx.c_str());
    e.l("s_mov_b64 exec, s[68:69]");
    e.l("v_add_u32_e32 %s, 0x%x, %s", e.v(x), uint32_t(sl.d * int32_t(j)), e.v(x));
    e.l("v_mov_b32 %s, %s", e.v(y), T[j - 1]);
    if (slot.first >= 0) {   // (the load cache: the word that ended the scan, and its address)
      e.l("v_add_u32_e32 v%d, 0x%x, %s", slot.first, sl.off, e.v(x));
      e.l("v_mov_b32 v%d, %s", slot.second, T[j - 1]);
    }
    e.l("v_add_u32_e32 %s, 0x%x, %s", VCNT, uint32_t(int32_t(j * r.cnt) + int32_t(j - 1) * tcnt), VCNT);
    e.l("v_mov_b32 %s, 0x%x", VPC, fall);
    if (!fall_in) e.l("s_or_b64 s[76:77], s[76:77], exec");   // (waits outside the trips)
    e.l("s_mov_b64 exec, s[82:83]");
    e.l("%s:", nx.c_str());
  }
  // still looping after U iterations: round again in the next trip
  e.l("s_mov_b64 exec, s[82:83]");
  e.l("s_cbranch_execz %s_sb", L.c_str());
  e.l("v_add_u32_e32 %s, 0x%x, %s", e.v(x), uint32_t(sl.d * int32_t(U)), e.v(x));
  e.l("v_mov_b32 %s, %s", e.v(y), T[U - 1]);
  e.l("v_add_u32_e32 %s, 0x%x, %s", VCNT, uint32_t(int32_t(U) * (int32_t(r.cnt) + tcnt)), VCNT);
  e.l("%s_sb:", L.c_str());
  e.l("s_mov_b64 exec, s[84:85]");
  e.l("s_cbranch_execz %s", e.stage_end.c_str());
}

// a run whose RET record POST_CALL may read along (Em::ret_pf): first a POST_CALL that
// restores cells, last a RET (nothing in between moves the call stack)
bool ret_prefetch_run(const Program &P, const JitRun &r) {
  if (r.len < 2) return false;
  const DInstr &f = P.code[r.pc], &l = P.code[r.pc + r.len - 1];
  return op_of(f) == OP_POST_CALL && (f.w1 & 0xFFFFu) > P.global_cells && op_of(l) == OP_RET;
}

// hybrid: only the trips' code (Ltin, the trip loop, the runs' stages, the exits), for
// jit_source's SIMT code object, whose Lsched sends diverged waves to Ltin; a trip after
// which every lane is at one pc goes back to Lsched (SIMT scheduling, direct run-to-run
// jumps) -- converged phases (C3's fill and checksum loops; modules like mt19937 whose
// addresses merely look divergent to the static analysis) run without trips.
std::string trip_source(const Program &P, const std::vector<JitRun> &runs, uint32_t glog, bool hybrid) {
  std::map<uint32_t, size_t> start;
  for (size_t k = 0; k < runs.size(); k++) start[runs[k].pc] = k;
  auto in_region = [&](uint32_t pc) { return start.count(pc) != 0; };
  // the pcs a return of function f can land on: after each direct call of f and after
  // every call_indirect
  std::map<uint32_t, uint32_t> fentry;
  for (uint32_t f = 0; f < P.funcs.size(); f++)
    if (!P.funcs[f].imported) fentry[P.funcs[f].entry_pc] = f;
  auto func_of = [&](uint32_t pc) -> int64_t {
    auto it = fentry.upper_bound(pc);
    return it == fentry.begin() ? -1 : int64_t(std::prev(it)->second);
  };
  std::map<int64_t, std::vector<uint32_t>> ret_out;   // function -> return pcs outside the runs
  std::vector<uint32_t> ind_out;
  for (uint32_t pc = 0; pc + 1 < P.code.size(); pc++) {
    const uint16_t o = op_of(P.code[pc]);
    if (o == OP_CALL && !in_region(pc + 1)) ret_out[func_of(P.code[pc].w3)].push_back(pc + 1);
    if (o == OP_CALL_INDIRECT && !in_region(pc + 1)) ind_out.push_back(pc + 1);
  }
  std::string body;
  if (!hybrid)
    body += "s_getpc_b64 s[6:7]\nLpt:\ns_add_u32 s6, s6, Ltab - Lpt\ns_addc_u32 s7, s7, 0\n"
            "s_mov_b32 %0, s6\ns_mov_b32 %1, s7\n"
            "s_getpc_b64 s[8:9]\nLpe:\ns_add_u32 s8, s8, Lend - Lpe\ns_addc_u32 s9, s9, 0\n"
            "s_setpc_b64 s[8:9]\n";
  Em h;   // entry stubs, the trip loop and its exits
  // a run's entry (its TInstr): the group's lanes record their pc and count; then every
  // lane's place is sorted out (OUTSIDE: not at a run start) and the trips begin
  // (hybrid: the runs' TInstrs enter their SIMT code; Lsched enters the trips)
  for (size_t k = 0; k < runs.size() && !hybrid; k++) {
    h.l(".p2align 6");   // (jit_load expects 64-byte aligned run addresses)
    h.l("Lb%zu:", k);
    h.l("v_lshrrev_b32_e64 %s, 5, s62", VPC);
    flush(h);
    long_jump(h, "Ltin", "Ltiq" + std::to_string(k));
  }
  // ---- the load cache (WB_TRIP_FWD=0 turns it off). A lane's scan that ends leaves the
  // word it ended on and that word's address in VGPRs above the frame (a slot per scan
  // run); a later run of the same trip loop whose every stage-A load is a 32-bit load at a
  // slot's address (C3's swap re-reads a[i] and a[j], which the two Hoare scans just ended
  // on) runs, for the lanes that arrived at it in this trip and whose addresses match, in
  // this same trip, its loads as moves -- instead of waiting for the next trip's stage A.
  // A slot is invalid (-1) from the trips' entry (Ltin: code outside the trips may have
  // stored), from its scan's stage A, and after any store of the lane (emit_store).
  const bool fwd_on = !(getenv("WB_TRIP_FWD") && getenv("WB_TRIP_FWD")[0] == '0');
  std::vector<std::pair<int, int>> slot_of(runs.size(), {-1, -1});
  // granule_addr's constant (Em::madk) in v255 when the first memory stays below kMadPages
  // (WB_TRIP_MAD=0: the 64-bit form); the slots below it
  const bool mad_on = g_mem_pages <= kMadPages && P.has_mem && 128 + 2 * P.total_cells() + 16 < 255 &&
                      !(getenv("WB_TRIP_MAD") && getenv("WB_TRIP_MAD")[0] == '0');
  const uint32_t top = mad_on ? 254 : 255;
  std::vector<uint32_t> slot_regs;   // address VGPRs
  {
    uint32_t ns = 0;
    for (size_t k = 0; k < runs.size(); k++) {
      ScanLoop sl;
      if (!fwd_on || !scan_loop_of(P, runs[k], &sl)) continue;
      const int a = int(top) - 2 * int(ns), v = a - 1;
      // (above the frame, above what inlined callees may use of it, never the frame's)
      if (uint32_t(v) < 128 + 2 * P.total_cells() + 16) break;
      slot_of[k] = {a, v};
      slot_regs.push_back(uint32_t(a));
      ns++;
    }
  }
  std::string ooa, oob;   // the runs' stage code, out of line
  std::vector<uint32_t> split(runs.size());
  const uint32_t nr = uint32_t(runs.size());
  // (A/B and debugging aids: WB_TRIP_SPLIT=0 runs every run whole in stage B;
  // WB_JIT_SCHED=0 keeps program order)
  const bool split_on = !(getenv("WB_TRIP_SPLIT") && getenv("WB_TRIP_SPLIT")[0] == '0');
  const bool sched_on = !(getenv("WB_JIT_SCHED") && getenv("WB_JIT_SCHED")[0] == '0');
  const bool nob_on = !(getenv("WB_NANOBS") && getenv("WB_NANOBS")[0] == '0');
  const std::vector<uint8_t> nob = nob_on ? nan_observable(P) : std::vector<uint8_t>();
  const bool ret_pf_on = !(getenv("WB_RET_PF") && getenv("WB_RET_PF")[0] == '0');
  const bool brt_on = !(getenv("WB_BRT_THREAD") && getenv("WB_BRT_THREAD")[0] == '0');
  for (uint32_t k = 0; k < nr && split_on; k++) {
    const JitRun &r = runs[k];
    const uint16_t lop = op_of(P.code[r.pc + r.len - 1]);
    split[k] = trip_split(P, r, ends_run(lop) ? r.len - 1 : r.len);
  }
  // Scan loops (scan_loop_of: `x += d; y = load(x + off); br y CMP p` back to the run's
  // start) run kTripScan iterations per trip: stage A checks the whole window of kTripScan
  // addresses once per lane and loads them all; stage B finds each lane's exit iteration
  // in order. A lane whose window fails the check (near its memory's end) takes the plain
  // one-iteration path, which meets a failing access exactly. WB_TRIP_SCAN=0 turns it off.
  const char *tse = getenv("WB_TRIP_SCAN");
  const uint32_t scan_k = tse ? std::min<uint32_t>(uint32_t(atoi(tse)), kTripScan) : kTripScan;
  std::vector<ScanLoop> scans(nr);
  std::vector<uint8_t> is_scan(nr, 0);
  for (uint32_t k = 0; k < nr && scan_k >= 2; k++)
    is_scan[k] = split[k] == 2 && scan_loop_of(P, runs[k], &scans[k]);
  for (uint32_t k = 0; k < nr; k++)
    if (!is_scan[k]) slot_of[k] = {-1, -1};   // (its cache slot is never set: unused)
  // the load cache's consumers: runs with a stage A of 32-bit loads at scan slots only
  std::vector<std::map<uint32_t, std::pair<uint32_t, uint32_t>>> fwd(nr);
  std::vector<uint8_t> fwd_ok(nr, 0);
  for (uint32_t k = 0; k < nr && !slot_regs.empty(); k++) {
    if (!split[k] || is_scan[k]) continue;
    bool ok = true, any = false;
    for (uint32_t i = 0; i < split[k] && ok; i++) {
      const DInstr &I = P.code[runs[k].pc + i];
      const uint16_t op = op_of(I);
      if (!mem_bytes(op) && !xmop(I)) continue;
      ok = false;
      const bool xl = op == OP_XLD && xmop(I) == OP_LD32;
      if (op != OP_LD32 && !xl) break;
      const uint32_t mk = xl ? (I.w1 >> 16) : 0;   // (the cache holds its scan's memory's words)
      for (uint32_t q = 0; q < nr; q++)
        if (is_scan[q] && slot_of[q].first >= 0 && scans[q].mem == mk && scans[q].x == (I.w1 & 0xFFFFu) &&
            scans[q].off == I.w3) {
          fwd[k][runs[k].pc + i] = {uint32_t(slot_of[q].first), uint32_t(slot_of[q].second)};
          ok = any = true;
          break;
        }
    }
    fwd_ok[k] = ok && any;
  }
  // the successor-window prefetch (trip_scan_prefetch; WB_TRIP_PF=0 turns it off):
  // pf_to[q] = the scan run scan q falls into, pf_from[s] = q
  const bool pf_on = !(getenv("WB_TRIP_PF") && getenv("WB_TRIP_PF")[0] == '0');
  std::vector<int> pf_to(nr, -1), pf_from(nr, -1);
  std::vector<ScanPrefetch> pfr(nr);
  std::vector<uint32_t> inval = slot_regs;   // (what a store invalidates: Em::inval)
  {
    uint32_t next = top - 2 * uint32_t(slot_regs.size());   // below the cache slots
    for (uint32_t q = 0; q < nr && pf_on && scan_k >= 2; q++) {
      if (!is_scan[q] || !start.count(runs[q].pc + 3)) continue;
      const uint32_t s = uint32_t(start[runs[q].pc + 3]);
      if (s == q || !is_scan[s] || pf_from[s] >= 0) continue;
      // (x in `next`, the window below it from an even register in address order: one
      // 16-byte load can fill it, scan_window_loads)
      const uint32_t lo = (next - scan_k) & ~1u;
      if (lo < 128 + 2 * P.total_cells() + 16) break;   // (as the slots)
      pfr[q].x = next;
      for (uint32_t j = 0; j < scan_k; j++)
        pfr[q].v.push_back("v" + std::to_string(scans[s].d < 0 ? lo + scan_k - 1 - j : lo + j));
      next = lo - 1;
      pf_to[q] = int(s);
      pf_from[s] = int(q);
      inval.push_back(pfr[q].x);
    }
  }
  h.l(".p2align 6");
  h.l("Ltin:");
  h.l("s_waitcnt lgkmcnt(0)");   // (a handler's bank-B prefetch must land: the batches use s[86:91])
  h.l("s_mov_b64 exec, s[96:97]");
  for (uint32_t r : inval) h.l("v_mov_b32 v%u, -1", r);
  if (mad_on) h.l("v_mov_b32 v255, 0x%x", 63u << (2 + glog));
  h.l("s_mov_b64 s[76:77], s[96:97]");
  h.l("s_mov_b64 s[78:79], 0");
  for (const auto &r : runs) {
    h.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", r.pc, VPC);
    h.l("s_andn2_b64 s[76:77], s[76:77], vcc");
  }
  // TPC for the next trip: the pc of every lane in the runs, -1 outside
  h.l("Ltp:");
  h.l("s_mov_b64 exec, s[96:97]");
  h.l("v_cndmask_b32_e64 %s, %s, -1, s[76:77]", TPC, VPC);
  // ---- the trip (EXEC = ALL between the runs)
  h.l("Ltrip:");
  // Batched lane tests (WB_TRIP_BATCH=0 turns them off): a run's test is a VALU compare
  // whose mask a scalar branch reads, and that VALU -> SALU -> branch chain costs ~48
  // cycles against ~20 for the branch alone (tools/ubench/lat.hip). So the compares of up
  // to kTripBatch consecutive tests go out back to back into their own masks (s[80:81],
  // s[86:91]: free between the runs; the trips start after every SMEM load has landed),
  // and the tests then read them. A stage-A run moves no other run's lanes (it only takes
  // its own out of TPC), so its batch stays valid; a stage-B run may move lanes onto later
  // runs (VPC), so it recomputes the rest of its batch before it returns (stage end), and a
  // run with its own LtF / LtS tests ends a batch.
  const bool batch_on = !(getenv("WB_TRIP_BATCH") && getenv("WB_TRIP_BATCH")[0] == '0');
  // Inline stages (WB_TRIP_INLINE=0 turns it off): a run's stage code sits in the test
  // chain right after its test, which branches past it when no lane is there -- a stage
  // that takes lanes costs no taken branch (out of line it costs two: there and back), one
  // that takes none costs one. Taken branches are what the trips' scalar stream waits on (a
  // taken branch refetches: ~20 cycles, tools/ubench/lat.hip); C3 1 MiB +6% with stage B
  // inline (profiles/r06zb_bench_c3_*).
  const bool inline_on = !(getenv("WB_TRIP_INLINE") && getenv("WB_TRIP_INLINE")[0] == '0');
  const bool smask_on = !(getenv("WB_TRIP_SMASK") && getenv("WB_TRIP_SMASK")[0] == '0');
  const bool cmpbr_on = !(getenv("WB_TRIP_CMPBR") && getenv("WB_TRIP_CMPBR")[0] == '0');
  // dst = (v == pc) per lane; VOP3 takes no literal, so a pc past the inline constants goes
  // through s68 / s69 (alternating: the compare has read one before the next is written)
  auto vcmp64 = [](Em &x, const char *dst, uint32_t pc, const char *v, uint32_t j) {
    if (pc <= 64) {
      x.l("v_cmp_eq_u32_e64 %s, %u, %s", dst, pc, v);
    } else {
      x.l("s_mov_b32 s%u, 0x%x", 68 + (j & 1), pc);
      x.l("v_cmp_eq_u32_e64 %s, s%u, %s", dst, 68 + (j & 1), v);
    }
  };
  static const char *const PREG[kTripBatch] = {"s[80:81]", "s[86:87]", "s[88:89]", "s[90:91]"};
  const uint32_t G = batch_on ? kTripBatch : 1;
  {
    std::vector<uint32_t> a;
    for (uint32_t k = 0; k < nr; k++)
      if (split[k]) a.push_back(k);
    for (size_t b = 0; b < a.size(); b += G) {
      const size_t e = std::min(a.size(), b + G);
      if (batch_on)
        for (size_t j = b; j < e; j++) vcmp64(h, PREG[j - b], runs[a[j]].pc, TPC, uint32_t(j - b));
      for (size_t j = b; j < e; j++) {
        if (batch_on) {
          h.l("s_and_b64 s[74:75], %s, exec", PREG[j - b]);
        } else {
          h.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", runs[a[j]].pc, TPC);
          h.l("s_and_b64 s[74:75], vcc, exec");
        }
        h.l("@@LtA%u@@", a[j]);   // (the test's branch and, inline, the stage-A code: below)
        h.l("LtAr%u:", a[j]);
      }
    }
  }
  h.l("s_waitcnt vmcnt(0)");
  // Forward chaining (WB_TRIP_CHAIN=0 turns it off): a run without a stage A takes every
  // lane now at its start -- the lanes that began the trip there and those an earlier
  // run of this trip moved there -- except the lanes waiting outside the trips (escapes
  // included). A run with a stage A takes only the lanes that began the trip there.
  const bool chain = !(getenv("WB_TRIP_CHAIN") && getenv("WB_TRIP_CHAIN")[0] == '0');
  // stage-B batches: run k's test reads PREG[k - bfirst[k]]; a stage-B run k recomputes
  // the masks of runs k+1 .. blast[k] (trip_source's stage code, below)
  // Guards (WB_TRIP_GUARD=0 turns them off): a block of consecutive runs is skipped after
  // one range test while no lane's VPC lies in its pc range (none of its tests could take
  // lanes then). The blocks: (1) the runs of one function -- C3's `sort` (fill and checksum
  // loops) while every lane sorts -- unless they are every run of the trips (a lane is
  // always in them then: C4's one function); (2) within those, a stretch of runs outside
  // every loop (no backward branch spans them: entries, exits, the trap tails after C4's
  // state machine), cold while the lanes loop. A block needs at least kTripGuard runs; the
  // test uses the batch registers and s68 / s69 where the block starts (after the runs
  // before it moved their lanes), blocks nest, and batches never cross a block's edge.
  // (VPC alone decides: a lane that a stage-B test takes by its TPC began the trip at that
  // run's pc and is still there -- a stage-A run moves none of its lanes but the ones that
  // leave, which take TPC -1, and no other run's test takes it.)
  const bool guard_on = batch_on && !(getenv("WB_TRIP_GUARD") && getenv("WB_TRIP_GUARD")[0] == '0');
  std::vector<int64_t> fn_of(nr);
  for (uint32_t k = 0; k < nr; k++) fn_of[k] = func_of(runs[k].pc);
  std::vector<uint8_t> in_loop(nr, 0);   // some backward branch spans the run's start
  for (uint32_t pc = 0; pc < P.code.size(); pc++) {
    const DInstr &I = P.code[pc];
    const uint16_t o = op_of(I);
    std::vector<uint32_t> tg;
    if (is_branch_op(o) || o == OP_BR_IF_MOV1 || o == OP_BR_IF_MOV2) tg.push_back(I.w3);
    if (o == OP_BR_TABLE)
      for (uint32_t q = 0; q <= (I.w1 >> 16); q++)
        if (2 * (size_t(I.w3) + q) < P.brtab.size()) tg.push_back(P.brtab[2 * (size_t(I.w3) + q)]);
    for (uint32_t t : tg)
      if (t <= pc)
        for (uint32_t k = 0; k < nr; k++) in_loop[k] |= runs[k].pc >= t && runs[k].pc <= pc;
  }
  std::vector<std::vector<uint32_t>> gblk(nr);   // block start -> the last runs of its blocks (outer first)
  std::vector<uint8_t> cut(nr + 1, 0);            // a block's edge lies before run k
  auto add_block = [&](uint32_t k, uint32_t e) {
    if (e + 1 - k < kTripGuard) return;
    gblk[k].push_back(e);
    cut[k] = cut[e + 1] = 1;
  };
  for (uint32_t k = 0; k < nr && guard_on;) {
    uint32_t e = k;
    while (e + 1 < nr && fn_of[e + 1] == fn_of[k]) e++;
    if (!(k == 0 && e + 1 == nr)) add_block(k, e);
    for (uint32_t j = k; j <= e;) {   // the function's stretches outside every loop
      if (in_loop[j]) { j++; continue; }
      uint32_t f = j;
      while (f + 1 <= e && !in_loop[f + 1]) f++;
      if (!(j == k && f == e)) add_block(j, f);   // (not the function's block again)
      j = f + 1;
    }
    k = e + 1;
  }
  std::vector<uint32_t> bfirst(nr, 0), blast(nr, 0);
  for (uint32_t k = 0; k < nr;) {
    uint32_t e = k;
    while (e + 1 < nr && e + 1 - k < G && !fwd_ok[e] && pf_from[e] < 0 && !cut[e + 1]) e++;
    for (uint32_t j = k; j <= e; j++) { bfirst[j] = k; blast[j] = e; }
    k = e + 1;
  }
  auto b_cmp = [&](Em &x, uint32_t k) {   // run k's test mask into its batch register
    vcmp64(x, PREG[k - bfirst[k]], runs[k].pc, chain && !split[k] ? VPC : TPC, k - bfirst[k]);
  };
  std::vector<std::pair<uint32_t, uint32_t>> gopen;   // (label id, last run) of blocks still open
  uint32_t nguard = 0;
  for (uint32_t k = 0; k < nr; k++) {
    for (uint32_t e : gblk[k]) {   // lo <= VPC <= hi (VPC - lo <= hi - lo), else past the block
      const uint32_t lo = runs[k].pc, hi = runs[e].pc;
      if (lo) {
        h.l("v_subrev_u32_e32 %s, 0x%x, %s", X0, lo, VPC);
        h.l("v_cmp_ge_u32_e32 vcc, 0x%x, %s", hi - lo, X0);
      } else {
        h.l("v_cmp_ge_u32_e32 vcc, 0x%x, %s", hi, VPC);
      }
      h.l("s_cbranch_vccz Lg%u", nguard);
      gopen.push_back({nguard++, e});
    }
    if (batch_on && bfirst[k] == k)
      for (uint32_t j = k; j <= blast[k]; j++) b_cmp(h, j);
    if (batch_on) {
      if (chain && !split[k]) h.l("s_andn2_b64 s[74:75], %s, s[76:77]", PREG[k - bfirst[k]]);
      else h.l("s_and_b64 s[74:75], %s, exec", PREG[k - bfirst[k]]);
    } else if (chain && !split[k]) {
      h.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", runs[k].pc, VPC);
      h.l("s_andn2_b64 s[74:75], vcc, s[76:77]");
    } else {
      h.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", runs[k].pc, TPC);
      h.l("s_and_b64 s[74:75], vcc, exec");
    }
    h.l("@@LtB%u@@", k);   // (the test's branch and, inline, the stage-B code: below)
    h.l("LtBr%u:", k);
    if (fwd_ok[k]) {   // the lanes that arrived this trip (not at its start there): LtF
      h.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", runs[k].pc, VPC);
      h.l("s_andn2_b64 s[74:75], vcc, s[76:77]");
      h.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", runs[k].pc, TPC);
      h.l("s_andn2_b64 s[74:75], s[74:75], vcc");
      h.l("@@LtF%u@@", k);
      h.l("LtFr%u:", k);
    }
    if (pf_from[k] >= 0) {   // the lanes its prefetching scan moved here this trip: LtS
      h.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", runs[k].pc, VPC);
      h.l("s_andn2_b64 s[74:75], vcc, s[76:77]");
      h.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", runs[k].pc, TPC);
      h.l("s_andn2_b64 s[74:75], s[74:75], vcc");
      h.l("@@LtS%u@@", k);
      h.l("LtSr%u:", k);
    }
    while (!gopen.empty() && gopen.back().second == k) {
      h.l("Lg%u:", gopen.back().first);
      gopen.pop_back();
    }
  }
  // ---- after the trip: go on while more lanes are in the runs than outside them (Ltnc;
  // none in the runs implies more outside than in, since ALL is not empty). The common
  // case -- every lane in the runs, at more than one pc -- falls through to the budget and
  // takes one branch, back to Ltp.
  h.l("s_cmp_eq_u64 s[76:77], 0");
  h.l("s_cbranch_scc0 Ltnc");
  // every lane in the runs and at one pc: back to SIMT scheduling (hybrid; Ltck). The test
  // (a VALU -> SGPR -> VALU -> branch chain) runs after every 16th trip only: CNT (s65, 0
  // in the trips: nothing in them counts through it) counts trips in its top four bits and
  // carries back to 0 on the 16th (WB_TRIP_CONV1=1: every trip; WB_TRIP_CONVP=k: every
  // 2^k-th, k = 1..8). C4 kernel 1.36e12 (every trip) -> 1.60e12 (2nd) -> 1.69e12 (4th) ->
  // 1.76e12 (8th) -> 1.82e12 (16th) -> 1.80e12 (64th); C3 and mt unchanged
  // (`profiles/r06zl_*`, `r06zo_*`): a wave whose last lanes stand at one pc no longer
  // leaves the trips for SIMT scheduling and re-enters them at the next split, trip
  // after trip (each entry re-marks the lanes outside the runs, one compare per run).
  const bool conv_every = getenv("WB_TRIP_CONV1") && getenv("WB_TRIP_CONV1")[0] == '1';
  const char *cpe = getenv("WB_TRIP_CONVP");
  const uint32_t conv_log = cpe ? std::min(8u, std::max(1u, uint32_t(atoi(cpe)))) : 4u;
  if (hybrid && !conv_every) {
    h.l("s_add_u32 s65, s65, 0x%x", 1u << (32 - conv_log));
    h.l("s_cbranch_scc1 Ltck");
  } else if (hybrid) {
    h.l("s_branch Ltck");
  }
  h.l("Ltbud:");
  // (>= what one lane can retire in a trip: one run, or with chaining every run once)
  uint32_t trip_cost = 256, chained = 0;
  for (uint32_t k = 0; k < nr; k++) {
    const JitRun &r = runs[k];
    trip_cost = std::max(trip_cost, r.cnt);
    chained += (fwd_ok[k] ? 2 : 1) * (r.cnt + 64);   // (+ a taken branch's correction)
    if (is_scan[k]) {
      const uint32_t sc = scan_k * uint32_t(std::max<int32_t>(
                                       0, int32_t(r.cnt) + int16_t(P.code[r.pc + 2].w2 >> 16))) + r.cnt;
      trip_cost = std::max<uint32_t>(trip_cost, sc);
      if (pf_from[k] >= 0) chained += sc + 64;   // (LtS: a whole window in the same trip)
    }
  }
  if (chain) trip_cost = std::max(trip_cost, chained + (uint32_t)kTripScan * 64u);
  // (no borrow: go on -- a budget that reaches 0 exactly runs one more trip)
  h.l("s_sub_u32 s64, s64, 0x%x", trip_cost);
  h.l("s_cbranch_scc0 Ltp");
  // budget spent: back to the kernel with no group (reason 1)
  h.l("s_mov_b32 s64, 0");
  h.l("s_mov_b64 exec, 0");
  h.l("s_mov_b32 s65, 0");
  h.l("s_add_u32 s68, s70, %u", TC_JIT_XS);
  h.l("s_addc_u32 s69, s71, 0");
  h.l("s_setpc_b64 s[68:69]");
  if (hybrid) {
    h.l("Ltck:");
    h.l("v_readfirstlane_b32 s68, %s", VPC);
    h.l("s_nop 1");
    h.l("v_cmp_ne_u32_e64 vcc, s68, %s", VPC);
    h.l("s_cbranch_vccnz Ltbud");
    h.l("s_mov_b32 s65, 0");   // (0 already unless WB_TRIP_CONV1)
    long_jump(h, "Lsched", "Ltcq");
  }
  // Ltnc: some lanes outside the runs. The wave leaves the trips (Ltx) only when more
  // than 64 times as many are outside as in -- i.e. when none is in: the lanes outside
  // (C4's finished state machines at its trap tails) wait and then run their code together,
  // instead of the wave leaving and re-entering the trips whenever they outnumber the rest
  // (WB_TRIP_OUTSH=k: more than 2^k times as many, k = 0..6; C4 kernel 1.67e12 at k = 0 ->
  // 1.79 (1) -> 1.83 (2) -> 1.86 (3) -> 1.91 (4) -> 2.03e12 (6) per step, C3 and mt
  // unchanged: `profiles/r06zu_*`, `r06zv_*`). Lanes outside are never stranded: a budget
  // exit hands the wave back to the kernel's scheduler, which picks among every lane.
  const char *ose = getenv("WB_TRIP_OUTSH");
  const int out_sh = ose ? std::max(0, std::min(6, atoi(ose))) : 6;
  h.l("Ltnc:");
  h.l("s_andn2_b64 s[80:81], s[96:97], s[76:77]");
  h.l("s_bcnt1_i32_b64 s68, s[80:81]");
  h.l("s_bcnt1_i32_b64 s69, s[76:77]");
  if (out_sh) h.l("s_lshl_b32 s68, s68, %d", out_sh);
  h.l("s_cmp_gt_u32 s69, s68");
  h.l("s_cbranch_scc0 Ltbud");
  // ---- leaving the trips: escapes first (the C++ step executes their instruction: xh),
  // then the other lanes outside (their handlers, through the scheduler's pick)
  h.l("Ltx:");
  h.l("s_cmp_eq_u64 s[78:79], 0");
  h.l("s_cbranch_scc1 Ltq");
  h.l("s_mov_b64 exec, -1");
  h.l("s_mov_b64 s[74:75], s[78:79]");
  h.l("s_nop 4");
  wave_min_vpc(h, "s[74:75]", "s68");
  h.l("s_lshl_b32 s62, s68, 5");
  h.l("v_cmp_eq_u32_e64 vcc, s68, %s", VPC);
  h.l("s_and_b64 s[74:75], vcc, s[74:75]");
  h.l("s_andn2_b64 vcc, s[96:97], s[74:75]");
  h.l("s_mov_b32 s63, -1");
  h.l("s_cbranch_vccz Ltxg");
  wave_min_vpc(h, "vcc", "s63");
  h.l("s_lshl_b32 s63, s63, 5");
  h.l("Ltxg:");
  h.l("s_mov_b32 s95, s63");
  h.l("s_mov_b32 s65, 0");
  h.l("s_mov_b64 exec, s[74:75]");
  h.l("s_setpc_b64 s[70:71]");
  h.l("Ltq:");
  h.l("s_mov_b32 s65, 0");   // (the trip count of Ltck)
  sched_block(h, "Ltq", "s[76:77]");
  // ---- the runs' stages
  for (uint32_t k = 0; k < nr; k++) {
    const JitRun &r = runs[k];
    const DInstr &last = P.code[r.pc + r.len - 1];
    const uint16_t lop = op_of(last);
    const uint32_t nbody = ends_run(lop) ? r.len - 1 : r.len;
    std::vector<int> lead;
    const std::vector<MemGroup> groups = jit_groups(P, r, &lead);
    // Groups a stage need not test (MemGroup::checked): every access of the group a 32-bit
    // access at a (cell, offset) whose 32-bit access these lanes already passed the test
    // for, with the cell unwritten since the run's start -- in the load cache's stage (LtF)
    // the cached addresses (the scan windows that set them were tested), in stage B of a
    // run with a stage A the stage-A accesses (C3's swap stores at the words its stage A
    // loaded). WB_TRIP_FWDCHK=0 keeps every test.
    const bool skip_on = !(getenv("WB_TRIP_FWDCHK") && getenv("WB_TRIP_FWDCHK")[0] == '0');
    auto mark_checked = [&](std::vector<MemGroup> &gs, const std::vector<std::pair<uint32_t, uint32_t>> &ok,
                            uint32_t from) {
      std::vector<uint8_t> good(gs.size(), 1), written_c(TC_VF_CELLS + 8, 0);
      int cur = -1;
      std::vector<uint32_t> w;
      for (uint32_t i = 0; i < r.len; i++) {
        const DInstr &I = P.code[r.pc + i];
        const uint16_t op = op_of(I);
        if (lead[i] >= 0) cur = lead[i];
        if (const uint32_t n = mem_bytes(op)) {
          const uint32_t a = I.w1 & 0xFFFFu;
          const bool hit = std::find(ok.begin(), ok.end(), std::make_pair(a, I.w3)) != ok.end();
          if (cur >= 0 && (i < from || n != 4 || !hit || a >= written_c.size() || written_c[a]))
            good[size_t(cur)] = 0;
        } else if (xmop(I)) {
          cur = -1;
        }
        written(I, &w);
        for (uint32_t x : w)
          if (x < written_c.size()) written_c[x] = 1;
      }
      for (size_t q = 0; q < gs.size(); q++) gs[q].checked = good[q] != 0;
    };
    std::vector<MemGroup> groups_f = groups, groups_b = groups;
    if (skip_on && fwd_ok[k]) {
      std::vector<std::pair<uint32_t, uint32_t>> ok;
      for (const auto &f : fwd[k]) ok.push_back({P.code[f.first].w1 & 0xFFFFu, P.code[f.first].w3});
      mark_checked(groups_f, ok, 0);
    }
    if (skip_on && split[k] && !is_scan[k]) {
      std::vector<std::pair<uint32_t, uint32_t>> ok;
      for (uint32_t i = 0; i < split[k]; i++) {
        const DInstr &I = P.code[r.pc + i];
        if (mem_bytes(op_of(I)) == 4) ok.push_back({I.w1 & 0xFFFFu, I.w3});
      }
      mark_checked(groups_b, ok, split[k]);
    }
    uint32_t done = 0, done_a = 0;
    // st 0: stage A, 1: stage B, 2: the whole run for the lanes the load cache serves (LtF),
    // 3: stage B for the lanes whose window a prefetching scan loaded this trip (LtS)
    static const char *const stage_name[4] = {"LtA", "LtB", "LtF", "LtS"};
    for (int st = 0; st < 4; st++) {
      bool salu_moved = false;   // (the transfer joined its moved lanes to the batch: join_batch)
      if (st == 0 && !split[k]) continue;
      if (st == 2 && !fwd_ok[k]) continue;
      if (st == 3 && pf_from[k] < 0) continue;
      const int sb = st == 3 ? 1 : st;   // (the stage the code is)
      Em e;
      e.trip = true;
      if (mad_on) e.madk = "v255";
      e.inval = inval;
      if (st == 2) e.fwd = fwd[k];
      if (!nob.empty()) e.nanobs = &nob;
      if (ret_pf_on && ret_prefetch_run(P, r)) {   // (POST_CALL in stage A: RET reads v113 in B)
        e.ret_pf = true;
        e.ret_pf_done = sb == 1 && split[k] > 0;
      }
      e.g = glog;
      e.fb = P.global_cells;
      e.prog = &P;
      e.run = (hybrid ? 8 * nr : 0) + k + uint32_t(st) * nr;   // (labels apart from the SIMT runs')
      e.done = st == 2 ? 0 : st == 3 ? done_a : done;
      const std::string L = stage_name[st] + std::to_string(k);
      e.stage_end = L + "e";
      e.l(".p2align 2");
      e.l("%s:", L.c_str());
      e.l("s_mov_b64 exec, s[74:75]");
      if (st == 0 && pf_to[k] >= 0) trip_scan_prefetch(e, scans[size_t(pf_to[k])], scan_k, pfr[k], L);
      if (st == 3) {   // the lanes still at the prefetched x: the window as if loaded in stage A
        const ScanPrefetch &pf = pfr[size_t(pf_from[k])];
        e.l("v_cmp_eq_u32_e32 vcc, v%u, %s", pf.x, e.v(scans[k].x));
        e.l("s_and_b64 exec, exec, vcc");
        e.l("s_cbranch_execz %s", e.stage_end.c_str());
        if (!scan_bf_on()) {   // (the branch-free stage B reads the prefetch registers)
          for (uint32_t j = 0; j < scan_k; j++) e.l("v_mov_b32 %s, %s", scan_T(scans[k], j), pf.v[j].c_str());
          e.l("v_mov_b32 v112, 1");
        }
      }
      if (st == 2) {   // the lanes whose every cached word is at its load's address
        // (the effective address is 33 bits: a lane whose x + offset carries, or lands on
        // 0xFFFFFFFF -- the invalid slots' mark, never a 4-byte load in bounds -- takes
        // the plain path, which traps it)
        for (const auto &f : fwd[k]) {
          const DInstr &I = P.code[f.first];
          if (I.w3) {
            e.l("v_add_co_u32_e32 %s, vcc, 0x%x, %s", Y0, I.w3, e.v(I.w1 & 0xFFFFu));
            e.l("s_andn2_b64 exec, exec, vcc");
          } else {
            e.l("v_mov_b32 %s, %s", Y0, e.v(I.w1 & 0xFFFFu));
          }
          e.l("v_cmp_ne_u32_e32 vcc, -1, %s", Y0);
          e.l("s_and_b64 exec, exec, vcc");
          e.l("v_cmp_eq_u32_e32 vcc, v%u, %s", f.second.first, Y0);
          e.l("s_and_b64 exec, exec, vcc");
        }
        e.l("s_cbranch_execz %s", e.stage_end.c_str());
      }
      if (is_scan[k])
        trip_scan_stage(e, P, r, scans[k], scan_k, sb, in_region(r.pc + 3), L, slot_of[k],
                        st == 3 && scan_bf_on() ? &pfr[size_t(pf_from[k])].v : nullptr);
      const size_t at = e.o.size();
      const uint32_t i0 = sb == 1 ? split[k] : 0, i1 = st == 0 ? split[k] : nbody;
      for (uint32_t i = i0; i < i1; i++) {
        const DInstr &I = P.code[r.pc + i];
        e.pc = r.pc + i;
        e.group = lead[i] >= 0 ? &(st == 2 ? groups_f : st == 1 ? groups_b : groups)[size_t(lead[i])] : nullptr;
        if (!emit(e, I)) return "";
        e.done += (I.w0 >> 16) & 0xFFu;
      }
      if (st < 2) done = e.done;
      if (st == 0) done_a = e.done;
      if (st >= 1) {
        // (loads in flight land first: the transfer reads cells -- a branch's operands, a
        // call's spill, a return's results)
        e.drain();
        // the transfer, per lane: VPC = where each lane goes on, VCNT += what the run
        // retired (with a taken branch's count correction)
        const uint32_t fall = r.pc + r.len;
        const uint32_t tgt = (lop == OP_CALL || is_branch_op(lop)) ? last.w3 : 0;
        e.pc = r.pc + r.len - 1;
        e.group = nullptr;
        auto out_if = [&](const char *m) { e.l("s_or_b64 s[76:77], s[76:77], %s", m); };
        auto add_cnt = [&](int64_t c) { if (c) e.l("v_add_u32_e32 %s, 0x%x, %s", VCNT, uint32_t(c), VCNT); };
        // Lanes moved onto a later run of this run's test batch join that run's batch mask
        // by scalar ops on the mask that moved them (`m` is this run's EXEC, or VCC / ~VCC
        // under it: a "vcc" / "~vcc" in its place), instead of a compare the next test would
        // wait on (VALU -> SALU, ~28 cycles: tools/ubench/lat.hip). WB_TRIP_SMASK=0: compares.
        auto join_batch = [&](uint32_t to, const char *m) {
          if (st != 1 || !batch_on || !smask_on || is_scan[k]) return;   // (a scan's stage moves lanes itself)
          for (uint32_t j = k + 1; j <= blast[k]; j++) {
            if (runs[j].pc != to || split[j] || !chain) continue;
            const char *pr = PREG[j - bfirst[j]];
            if (m[0] == 'e') {   // ("exec")
              e.l("s_or_b64 %s, %s, exec", pr, pr);
            } else {
              e.l(m[0] == '~' ? "s_andn2_b64 s[68:69], exec, vcc" : "s_and_b64 s[68:69], vcc, exec");
              e.l("s_or_b64 %s, %s, s[68:69]", pr, pr);
            }
          }
        };
        // the run at pc when it is one br_table (a JMP onto it takes the table: WB_BRT_THREAD)
        auto brt_thread = [&](uint32_t pc) -> int {
          if (!brt_on || !start.count(pc)) return -1;
          const size_t q = start[pc];
          return runs[q].len == 1 && op_of(P.code[pc]) == OP_BR_TABLE ? int(q) : -1;
        };
        // the lanes a br_table sends out of the runs (Y0 = their targets)
        auto br_table_outs = [&](const DInstr &B) {
          std::vector<uint32_t> seen;
          for (uint32_t q = 0; q <= (B.w1 >> 16); q++) {
            const uint32_t t = P.brtab[2 * (B.w3 + q)];
            if (in_region(t) || std::find(seen.begin(), seen.end(), t) != seen.end()) continue;
            seen.push_back(t);
            e.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", t, Y0);
            e.l("s_and_b64 s[68:69], vcc, exec");
            out_if("s[68:69]");
          }
        };
        if (is_branch_op(lop) && lop != OP_JMP) {
          const int32_t tcnt = int32_t(int16_t(last.w2 >> 16));
          // A br_if / br_unless on the cell the run's last instruction set from VCC (a
          // compare: `v_cndmask cell, 0, 1, vcc` its last line, only waits after it) reads
          // VCC itself -- no compare of the cell again; br_unless then selects the other
          // way round (inv: VCC = not taken). WB_TRIP_CMPBR=0 compares again.
          bool inv = false, reuse = false;
          if ((lop == OP_BR_IF || lop == OP_BR_UNLESS) && cmpbr_on) {
            size_t end = e.o.size();
            while (end >= 2) {
              const size_t b0 = e.o.rfind('\n', end - 2);
              const size_t st0 = b0 == std::string::npos ? 0 : b0 + 1;
              const std::string ln = e.o.substr(st0, end - st0);
              if (ln.compare(0, 9, "s_waitcnt") == 0 || ln == "\n") { end = st0; continue; }
              reuse = ln == "v_cndmask_b32_e64 " + std::string(e.v(last.w1 & 0xFFFFu)) + ", 0, 1, vcc\n";
              break;
            }
          }
          if (!reuse) branch_cond(e, last);   // vcc = taken
          inv = reuse && lop == OP_BR_UNLESS;
          // (VOP3 selects take inline constants, -16..64: the pcs and corrections of small
          // modules need no moves)
          auto inl = [](int64_t v) { return v >= -16 && v <= 64; };
          std::string f = std::to_string(fall), t = std::to_string(tgt);
          if (!inl(fall)) { e.l("v_mov_b32 %s, 0x%x", X0, fall); f = X0; }
          if (!inl(tgt)) { e.l("v_mov_b32 %s, 0x%x", X1, tgt); t = X1; }
          if (inv) std::swap(f, t);
          e.l("v_cndmask_b32_e64 %s, %s, %s, vcc", VPC, f.c_str(), t.c_str());
          if (tcnt) {
            if (inl(tcnt)) {
              if (inv) e.l("v_cndmask_b32_e64 %s, %d, 0, vcc", X0, tcnt);
              else e.l("v_cndmask_b32_e64 %s, 0, %d, vcc", X0, tcnt);
            } else {
              e.l("v_mov_b32 %s, 0x%x", X1, uint32_t(tcnt));
              if (inv) e.l("v_cndmask_b32_e64 %s, %s, 0, vcc", X0, X1);
              else e.l("v_cndmask_b32_e32 %s, 0, %s, vcc", X0, X1);
            }
            if (r.cnt && inl(r.cnt)) {   // (the run's count in the same add)
              e.l("v_add3_u32 %s, %s, %s, %u", VCNT, VCNT, X0, r.cnt);
            } else {
              e.l("v_add_u32_e32 %s, %s, %s", VCNT, VCNT, X0);
              add_cnt(r.cnt);
            }
          } else {
            add_cnt(r.cnt);
          }
          const char *taken_m = inv ? "s_andn2_b64 s[68:69], exec, vcc" : "s_and_b64 s[68:69], vcc, exec";
          const char *fall_m = inv ? "s_and_b64 s[68:69], vcc, exec" : "s_andn2_b64 s[68:69], exec, vcc";
          if (!in_region(tgt)) { e.l("%s", taken_m); out_if("s[68:69]"); }
          if (!in_region(fall)) { e.l("%s", fall_m); out_if("s[68:69]"); }
          if (tgt == fall) {
            join_batch(tgt, "exec");
          } else {
            join_batch(tgt, inv ? "~vcc" : "vcc");
            join_batch(fall, inv ? "vcc" : "~vcc");
          }
          salu_moved = true;
        } else if (lop == OP_JMP && brt_thread(tgt) >= 0) {
          // a jump onto a run that is one br_table (C4's `br $machine` back to its state
          // dispatch): the table's choice made here, so that a lane whose entry lies ahead
          // in the run order goes on in this trip; a state set to a constant in this run
          // picks its entry at compile time. Counts: this run's, the jump's taken
          // correction, the br_table run's and its entry's correction.
          const DInstr &B = P.code[tgt];
          const uint32_t ba = B.w1 & 0xFFFFu, nb = B.w1 >> 16;
          add_cnt(int64_t(r.cnt) + int16_t(last.w2 >> 16) + runs[size_t(brt_thread(tgt))].cnt);
          int64_t kc = -1;   // the state cell's constant, if this run sets it last
          for (uint32_t i = nbody; i-- > 0;) {
            const DInstr &I = P.code[r.pc + i];
            std::vector<uint32_t> w;
            written(I, &w);
            if (std::find(w.begin(), w.end(), ba) == w.end()) continue;
            if (op_of(I) == OP_CONST32 && (I.w2 & 0xFFFFu) == ba) kc = I.w3;
            break;
          }
          if (kc >= 0) {
            const uint32_t q = std::min<uint32_t>(uint32_t(kc), nb);
            const uint32_t t = P.brtab[2 * (B.w3 + q)];
            e.l("v_mov_b32 %s, 0x%x", VPC, t);
            add_cnt(int32_t(P.brtab[2 * (B.w3 + q) + 1]));
            if (!in_region(t)) out_if("exec");
            join_batch(t, "exec");
            salu_moved = true;
          } else {
            emit_br_table(e, B);
            e.l("v_mov_b32 %s, %s", VPC, Y0);
            e.l("v_add_u32_e32 %s, %s, %s", VCNT, VCNT, Y1);
            br_table_outs(B);
          }
        } else if (lop == OP_JMP) {
          e.l("v_mov_b32 %s, 0x%x", VPC, tgt);
          add_cnt(int64_t(r.cnt) + int16_t(last.w2 >> 16));
          if (!in_region(tgt)) out_if("exec");
          join_batch(tgt, "exec");
          salu_moved = true;
        } else if (lop == OP_BR_TABLE) {
          emit_br_table(e, last);   // Y0 = target, Y1 = correction
          e.l("v_mov_b32 %s, %s", VPC, Y0);
          e.l("v_add_u32_e32 %s, %s, %s", VCNT, VCNT, Y1);
          add_cnt(r.cnt);
          br_table_outs(last);
        } else if (lop == OP_CALL) {
          std::vector<uint8_t> dead;
          if (start.count(tgt)) dead = dead_zeros(P, runs[start[tgt]]);
          emit_call(e, last, e.pc, dead.empty() ? nullptr : &dead);
          e.l("v_mov_b32 %s, 0x%x", VPC, tgt);
          add_cnt(r.cnt);
          if (!in_region(tgt)) out_if("exec");
        } else if (lop == OP_RET) {
          // per lane: the call stack past its LDS part and the entry function's return
          // leave (the C++ step); the others pop their own return record
          const uint32_t a = last.w1 & 0xFFFFu, nres = last.w1 >> 16, fb = e.fb;
          e.l("v_cmp_lt_u32_e64 %s, s93, v102", T2);
          e.leave_if_t2();
          if (e.ret_pf_done) {
            e.l("v_mov_b32 %s, v113", Y1);
          } else {
            e.l("v_lshl_add_u32 %s, v102, 8, v103", X1);
            e.l("v_subrev_u32_e32 %s, 0x100, %s", X1, X1);
            e.l("ds_read_b32 %s, %s", Y1, X1);
            e.l("s_waitcnt lgkmcnt(0)");
          }
          e.l("v_and_b32_e32 %s, 0xfffff, %s", X0, Y1);
          e.l("v_cmp_eq_u32_e32 vcc, 0xfffff, %s", X0);
          e.l("s_mov_b64 %s, vcc", T2);
          e.leave_if_t2();
          e.l("v_subrev_u32_e32 v102, 1, v102");
          for (uint32_t q = 0; q < nres; q++)
            if (a != fb) e.l("v_mov_b32 %s, %s", e.v(fb + q), e.v(a + q));
          e.l("v_mov_b32 %s, %s", VPC, X0);
          add_cnt(r.cnt);
          std::vector<uint32_t> outs = ind_out;
          const auto it = ret_out.find(func_of(e.pc));
          if (it != ret_out.end()) outs.insert(outs.end(), it->second.begin(), it->second.end());
          std::sort(outs.begin(), outs.end());
          outs.erase(std::unique(outs.begin(), outs.end()), outs.end());
          for (uint32_t t : outs) {
            e.l("v_cmp_eq_u32_e32 vcc, 0x%x, %s", t, X0);
            e.l("s_and_b64 s[68:69], vcc, exec");
            out_if("s[68:69]");
          }
        } else {   // falls through into the instruction after the run
          e.l("v_mov_b32 %s, 0x%x", VPC, fall);
          add_cnt(r.cnt);
          if (!in_region(fall)) out_if("exec");
          join_batch(fall, "exec");
          salu_moved = true;
        }
        e.drain();
      }
      std::string code = sched_on ? e.o.substr(0, at) + schedule(e.o.substr(at)) : e.o;
      code += e.stage_end + ":\n";
      code += "s_mov_b64 exec, s[96:97]\n";
      if (st == 1 && batch_on && !(smask_on && salu_moved && !is_scan[k])) {   // (moved lanes: the rest of its batch)
        // Only the tests of runs its lanes can go to: a test on TPC (a run with a stage A)
        // sees no move, and a run whose exits are known (a jump, a branch, falling through,
        // a jump onto a br_table's run) moves lanes only onto those pcs.
        std::vector<uint32_t> succ;
        bool known = !is_scan[k] && !fwd_ok[k] && pf_from[k] < 0 && pf_to[k] < 0;
        if (known) {
          const uint32_t fall = r.pc + r.len;
          if (lop == OP_JMP) {
            const int q = brt_on && start.count(last.w3) && runs[start[last.w3]].len == 1 &&
                                  op_of(P.code[last.w3]) == OP_BR_TABLE
                              ? int(start[last.w3]) : -1;
            if (q >= 0) {
              const DInstr &B = P.code[last.w3];
              for (uint32_t t = 0; t <= (B.w1 >> 16); t++) succ.push_back(P.brtab[2 * (B.w3 + t)]);
            } else {
              succ.push_back(last.w3);
            }
          } else if (is_branch_op(lop)) {
            succ = {fall, last.w3};
          } else if (!ends_run(lop)) {
            succ.push_back(fall);
          } else {
            known = false;
          }
        }
        Em rb;
        for (uint32_t j = k + 1; j <= blast[k]; j++) {
          if (known && (split[j] || std::find(succ.begin(), succ.end(), runs[j].pc) == succ.end())) continue;
          b_cmp(rb, j);
        }
        code += rb.o;
      }
      // the test's branch: past the stage inline (a stage short enough for the branch's
      // reach, 2^15 dwords: <= 2,048 lines of at most 12 bytes), else to it out of line
      const std::string mark = "@@" + L + "@@\n", ret = std::string(stage_name[st]) + "r" + std::to_string(k);
      const size_t at_m = h.o.find(mark);
      if (at_m == std::string::npos) return "";
      if (inline_on && std::count(code.begin(), code.end(), '\n') <= 2048) {
        const std::string al = ".p2align 2\n";   // (in the chain: no alignment)
        if (code.compare(0, al.size(), al) == 0) code.erase(0, al.size());
        h.o.replace(at_m, mark.size(), "s_cbranch_scc0 " + ret + "\n" + code);
        oob += e.tail;
        continue;
      }
      h.o.replace(at_m, mark.size(), "s_cbranch_scc1 " + L + "\n");
      code += "s_branch " + ret + "\n";
      code += e.tail;
      (st ? oob : ooa) += code;
    }
  }
  body += h.o + ooa + oob;
  if (hybrid) return body;
  body = resolve_jumps(body);
  body += ".p2align 3\nLtab:\n";
  for (size_t k = 0; k < runs.size(); k++) body += ".quad Lb" + std::to_string(k) + " - Ltab\n";
  body += "Lend:\n";
  std::string src =
      "// generated by jit.cpp: compiled runs of the V-frame threaded core (trip mode)\n"
      "extern \"C\" __global__ void wbjit_addrs(unsigned long long *out, unsigned n) {\n"
      "  unsigned lo, hi;\n"
      "  asm volatile(\n";
  for (size_t at = 0; at < body.size();) {
    const size_t nl = body.find('\n', at);
    src += "      \"" + body.substr(at, nl - at) + "\\n\"\n";
    at = nl + 1;
  }
  src += "      : \"=s\"(lo), \"=s\"(hi) : : \"s6\", \"s7\", \"s8\", \"s9\", \"scc\", \"memory\");\n"
         "  const long long *tab = (const long long *)(((unsigned long long)hi << 32) | lo);\n"
         "  for (unsigned k = threadIdx.x; k < n; k += blockDim.x)\n"
         "    out[k] = (unsigned long long)tab + (unsigned long long)tab[k];\n"
         "}\n";
  return src;
}

// ---------------------------------------------------------------- constant folding
// Cells read and written by the instructions the planner below lets stand between a fold
// and its uses: plain register ops that never leave the compiled code (no memory, no
// traps, no calls). Returns false for anything else.
bool pure_cells(const DInstr &I, std::vector<uint32_t> *rd, std::vector<uint32_t> *wr) {
  const uint16_t op = op_of(I);
  const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16, c = I.w2 & 0xFFFFu;
  auto R = [&](uint32_t x, uint32_t n) { for (uint32_t k = 0; k < n; k++) rd->push_back(x + k); };
  auto W = [&](uint32_t x, uint32_t n) { for (uint32_t k = 0; k < n; k++) wr->push_back(x + k); };
  switch (op) {
    case OP_V_F64X2_ADD: case OP_V_F64X2_SUB: case OP_V_F64X2_MUL: case OP_V_F64X2_EQ:
    case OP_V_F64X2_NE: case OP_V_F64X2_LT: case OP_V_F64X2_GT: case OP_V_F64X2_LE:
    case OP_V_F64X2_GE: case OP_V_I64X2_ADD: case OP_V_I64X2_SUB: case OP_V_I64X2_EQ:
      R(a, 4); R(b, 4); W(c, 4); return true;
    case OP_V_F64X2_SPLAT: case OP_V_I64X2_SPLAT: R(a, 2); W(c, 4); return true;
    case OP_V_ANY_TRUE: R(a, 4); W(c, 1); return true;
    case OP_V_EXTRACT64: R(a, 4); W(c, 2); return true;
    case OP_V_REPLACE64: R(a, 4); R(b, 2); W(c, 4); return true;
    case OP_CONST32: W(c, 1); return true;
    case OP_CONST64: W(c, 2); return true;
    case OP_CONST128: W(c, 4); return true;
    case OP_MOV32: R(a, 1); W(c, 1); return true;
    case OP_MOV64: R(a, 2); W(c, 2); return true;
    case OP_MOV128: R(a, 4); W(c, 4); return true;
    case OP_I32_ADD: case OP_I32_SUB: case OP_I32_AND: case OP_I32_OR: case OP_I32_XOR:
      R(a, 1); R(b, 1); W(c, 1); return true;
    case OP_I32_ADD_I: case OP_I32_SUB_I: case OP_I32_SHL_I: R(a, 1); W(c, 1); return true;
    case OP_I64_EXTEND_I32_U: case OP_F64_CONVERT_I32_U: case OP_F64_CONVERT_I32_S:
      R(a, 1); W(c, 2); return true;
    default: return false;
  }
}

// The f64 inline constants of a VOP3 operand (0 is left out: -0.0 is not one of them)
const char *f64_inline(uint64_t v) {
  switch (v) {
    case 0x3FE0000000000000ull: return "0.5";
    case 0xBFE0000000000000ull: return "-0.5";
    case 0x3FF0000000000000ull: return "1.0";
    case 0xBFF0000000000000ull: return "-1.0";
    case 0x4000000000000000ull: return "2.0";
    case 0xC000000000000000ull: return "-2.0";
    case 0x4010000000000000ull: return "4.0";
    case 0xC010000000000000ull: return "-4.0";
    default: return nullptr;
  }
}

// Per run: `CONST64 X, k; V_F64X2_SPLAT X -> X` where k is an inline constant and every
// later read of X..X+3 in the run is an f64x2 add/sub/mul/compare taking X as a whole
// operand (and whose NaN payload is never observed) is not materialized: those ops take
// k itself. X..X+3 must be written again later in the run or be dead where the run goes
// on (live: plain liveness, nan_observable), and nothing between the splat and the last
// use can leave the compiled code. C5: the 4.0 and 2.0 of its iteration (8 moves).
struct FoldPlan {
  std::vector<uint8_t> skip;                    // body index: not emitted
  std::map<uint32_t, std::vector<std::pair<uint32_t, std::string>>> at;   // body index -> (cell, constant)
};
FoldPlan plan_folds(const Program &P, const JitRun &r, uint32_t nbody,
                    const std::vector<std::vector<uint64_t>> &live, const std::vector<uint8_t> &nob,
                    const std::vector<LoadBatch> &batches) {
  FoldPlan fp;
  fp.skip.assign(r.len, 0);
  if (live.empty()) return fp;
  const DInstr &last = P.code[r.pc + r.len - 1];
  const uint16_t lop = op_of(last);
  std::vector<uint32_t> succ;
  if (nbody == r.len) succ.push_back(r.pc + r.len);
  else if (lop == OP_JMP) succ.push_back(last.w3);
  else if (is_branch_op(lop)) { succ.push_back(r.pc + r.len); succ.push_back(last.w3); }
  else return fp;   // (calls, returns, br_table: no folds)
  auto live_at = [&](uint32_t pc, uint32_t c) {
    return pc >= live.size() || (live[pc][c >> 6] >> (c & 63) & 1);
  };
  for (uint32_t i = 0; i + 1 < nbody; i++) {
    const DInstr &I = P.code[r.pc + i], &J = P.code[r.pc + i + 1];
    if (op_of(I) != OP_CONST64 || op_of(J) != OP_V_F64X2_SPLAT) continue;
    const uint32_t X = I.w2 & 0xFFFFu;
    if ((J.w1 & 0xFFFFu) != X || (J.w2 & 0xFFFFu) != X || uint64_t(X) + 4 > P.total_cells()) continue;
    const char *txt = f64_inline(uint64_t(I.w3) | (uint64_t(I.w1) << 32));
    if (!txt) continue;
    bool inbatch = false;
    for (const auto &b : batches) inbatch = inbatch || (b.i0 <= i + 1 && i < b.i1);
    if (inbatch) continue;
    std::vector<uint32_t> uses;
    bool ok = true, redefined = false;
    std::vector<uint8_t> cov(4, 0);   // cells of X..X+3 written again so far
    for (uint32_t j = i + 2; j < r.len && ok && !redefined; j++) {
      const DInstr &K = P.code[r.pc + j];
      const uint16_t ko = op_of(K);
      std::vector<uint32_t> rd, wr;
      if (j + 1 == r.len && nbody < r.len) {   // the run's branch
        const uint32_t ka = K.w1 & 0xFFFFu, kb = K.w1 >> 16;
        if (ko != OP_JMP && ka >= X && ka < X + 4 && !cov[ka - X]) ok = false;
        if (ko >= OP_BR_EQ && ko <= OP_BR_GE_U && kb >= X && kb < X + 4 && !cov[kb - X]) ok = false;
        break;
      }
      if (!pure_cells(K, &rd, &wr)) { ok = false; break; }
      const uint32_t ka = K.w1 & 0xFFFFu, kb = K.w1 >> 16, kc = K.w2 & 0xFFFFu;
      bool reads = false;   // (of a cell of X..X+3 still holding the constant)
      for (uint32_t x : rd) reads = reads || (x >= X && x < X + 4 && !cov[x - X]);
      bool overlap_w = false;
      for (uint32_t x : wr) overlap_w = overlap_w || (x >= X && x < X + 4);
      const bool arith = ko == OP_V_F64X2_ADD || ko == OP_V_F64X2_SUB || ko == OP_V_F64X2_MUL;
      const bool cmp = ko >= OP_V_F64X2_EQ && ko <= OP_V_F64X2_GE;
      const bool partly = cov[0] || cov[1] || cov[2] || cov[3];
      if (reads && partly) { ok = false; break; }
      if (reads) {
        const bool whole = (ka == X || kb == X) && !(ka != X && ka + 4 > X && ka < X + 4) &&
                           !(kb != X && kb + 4 > X && kb < X + 4);
        const bool quiet = !nob.empty() && r.pc + j < nob.size() && !nob[r.pc + j];
        // (a use whose result lands on X itself, in place, is the last: X is written again)
        if (!whole || (overlap_w && kc != X) || !((arith && quiet) || cmp)) { ok = false; break; }
        uses.push_back(j);
        if (overlap_w) redefined = true;
        continue;
      }
      if (overlap_w) {
        for (uint32_t x : wr) if (x >= X && x < X + 4) cov[x - X] = 1;
        if (cov[0] && cov[1] && cov[2] && cov[3]) redefined = true;
      }
    }
    if (!ok || uses.empty()) continue;
    if (!redefined)
      for (uint32_t t : succ)
        for (uint32_t q = 0; q < 4; q++) ok = ok && (cov[q] || !live_at(t, X + q));
    if (!ok) continue;
    fp.skip[i] = fp.skip[i + 1] = 1;
    for (uint32_t j : uses) {
      fp.at[j].push_back({X, txt});
      fp.at[j].push_back({X + 2, txt});
    }
    i++;
  }
  return fp;
}

// Whether a function can reach itself through calls: a cycle among direct calls (CALL,
// TAIL_CALL), or any indirect call (its targets are not known here)
bool recursive(const Program &P) {
  std::map<uint32_t, uint32_t> fentry;   // entry pc -> function
  for (uint32_t f = 0; f < P.funcs.size(); f++)
    if (!P.funcs[f].imported) fentry[P.funcs[f].entry_pc] = f;
  auto func_of = [&](uint32_t pc) -> int64_t {
    auto it = fentry.upper_bound(pc);
    return it == fentry.begin() ? -1 : int64_t(std::prev(it)->second);
  };
  const size_t nf = P.funcs.size();
  std::vector<std::vector<uint32_t>> g(nf);
  for (uint32_t pc = 0; pc < P.code.size(); pc++) {
    const uint16_t o = op_of(P.code[pc]);
    if (o == OP_CALL_INDIRECT || o == OP_TAIL_CALL_INDIRECT) return true;
    if (o != OP_CALL && o != OP_TAIL_CALL) continue;
    const int64_t a = func_of(pc), b = func_of(P.code[pc].w3);
    if (a < 0 || b < 0) continue;
    if (a == b) return true;
    g[size_t(a)].push_back(uint32_t(b));
  }
  std::vector<uint8_t> st(nf, 0);   // 0 new, 1 on the path, 2 done
  std::function<bool(uint32_t)> dfs = [&](uint32_t f) -> bool {
    st[f] = 1;
    for (uint32_t t : g[f]) {
      if (st[t] == 1) return true;
      if (st[t] == 0 && dfs(t)) return true;
    }
    st[f] = 2;
    return false;
  };
  for (uint32_t f = 0; f < nf; f++)
    if (st[f] == 0 && dfs(f)) return true;
  return false;
}

std::string jit_source(const Program &P, const std::vector<JitRun> &runs, uint32_t glog,
                       const JitCost *cost, bool simt, bool trip, const std::vector<uint32_t> *xinfo,
                       uint32_t xlog, uint32_t mem_pages) {
  if (cost) simt = false;
  // (extra memories: their accesses compile only against the context's word offsets)
  if (!P.xmems.empty() && (!xinfo || xinfo->size() < 2 * P.xmems.size())) return "";
  struct XinfoScope {
    XinfoScope(const std::vector<uint32_t> *x, uint32_t lg, uint32_t mp) { g_xinfo = x; g_xlog = lg; g_mem_pages = mp; }
    ~XinfoScope() { g_xinfo = nullptr; g_xlog = 0; g_mem_pages = 65536; }
  } xscope(xinfo, xlog, mem_pages);
  // trip mode beside SIMT scheduling (hybrid, the default) or alone (WB_HYBRID=0)
  const bool trips = trip && simt && runs.size() <= kTripMaxRuns;
  const bool hybrid = trips && !(getenv("WB_HYBRID") && getenv("WB_HYBRID")[0] == '0');
  if (trips && !hybrid) return trip_source(P, runs, glog, false);
  // NaN fixes only where the payload can be observed (WB_NANOBS=0: everywhere)
  const bool nob_on = !(getenv("WB_NANOBS") && getenv("WB_NANOBS")[0] == '0');
  const std::vector<uint8_t> nob = nob_on ? nan_observable(P) : std::vector<uint8_t>();
  // plain cell liveness (constant folds, fused any_true); WB_FOLD=0 turns both off
  std::vector<std::vector<uint64_t>> live;
  if (!(getenv("WB_FOLD") && getenv("WB_FOLD")[0] == '0')) nan_observable(P, &live);
  // an f64x2 compare feeding a fused any_true hands its lane masks to the branch (C5
  // 1.435e13 -> 1.475e13, profiles/r03ab_bench.json; WB_CMPANY=0 turns it off)
  const bool cmp_any_on = !(getenv("WB_CMPANY") && getenv("WB_CMPANY")[0] == '0');
  // which divergence events stay in the core (debug aid): 1 split branches, 2 split
  // returns, 4 reaching a waiting lane / the count limit (else the core leaves as without
  // SIMT)
  const char *sxe = getenv("WB_SIMT_X");
  const unsigned sx = simt ? (sxe ? unsigned(atoi(sxe)) : 7u) : 0u;
  const char *se = getenv("WB_JIT_SCHED");   // 0: keep program order (A/B measurement aid)
  const bool sched = !(se && se[0] == '0');
  const char *lbe = getenv("WB_LOAD_BATCH");   // 0: loads in program order (A/B aid)
  const bool batching = !(lbe && lbe[0] == '0');
  // One asm statement holds every run (behind a jump) and a table of their offsets from
  // the table itself; the kernel reads the table and writes the absolute addresses.
  std::string body;
  body += "s_getpc_b64 s[6:7]\nLpt:\ns_add_u32 s6, s6, Ltab - Lpt\ns_addc_u32 s7, s7, 0\n"
          "s_mov_b32 %0, s6\ns_mov_b32 %1, s7\n"
          "s_getpc_b64 s[8:9]\nLpe:\ns_add_u32 s8, s8, Lend - Lpe\ns_addc_u32 s9, s9, 0\n"
          "s_setpc_b64 s[8:9]\n";
  // Recursive modules pick groups by call-stack height first (sched_block); their split
  // branches go through that pick too (the pc-only shortcut, Lbf, would undo it).
  // WB_DEPTH=0: pc-only picks everywhere (A/B aid)
  const bool depth_pick = simt && !(getenv("WB_DEPTH") && getenv("WB_DEPTH")[0] == '0') &&
                          recursive(P);
  if (simt) body += simt_sched(hybrid, depth_pick);
  // run index by start pc: a transfer to one jumps straight to its code
  std::map<uint32_t, size_t> start;
  for (size_t k = 0; k < runs.size(); k++) start[runs[k].pc] = k;
  // a return's likely targets: the instruction after each direct call of its function
  // (functions are laid out in order of entry pc)
  std::map<uint32_t, uint32_t> fentry;   // entry pc -> function index
  for (uint32_t f = 0; f < P.funcs.size(); f++)
    if (!P.funcs[f].imported) fentry[P.funcs[f].entry_pc] = f;
  auto func_of = [&](uint32_t pc) -> int64_t {
    auto it = fentry.upper_bound(pc);
    return it == fentry.begin() ? -1 : int64_t(std::prev(it)->second);
  };
  std::map<uint32_t, std::vector<uint32_t>> ret_sites;   // function -> return pcs
  for (uint32_t pc = 0; pc < P.code.size(); pc++)
    if (op_of(P.code[pc]) == OP_CALL) {
      const int64_t f = func_of(P.code[pc].w3);
      if (f >= 0) ret_sites[uint32_t(f)].push_back(pc + 1);
    }
  // Inlined call: a leaf callee that is one compiled run ending in its return runs in
  // the calling run's code, its cells `off` = L - fb higher (above the caller's live
  // cells, which therefore need no spill), its arguments already in place at L.., its
  // result moved to L.., and the caller goes on after its POST_CALL (no call-stack
  // traffic, no return-record check). A leave inside the callee first makes the call real
  // (spill, return record, callee cells down to fb) so the C++ step meets the reference
  // layout. inline_of: the callee's run and the post-call run, or -1.
  const bool inl_env = !(getenv("WB_INLINE") && getenv("WB_INLINE")[0] == '0');
  auto inline_of = [&](size_t k, int64_t *inl_f, int64_t *inl_post) {
    *inl_f = *inl_post = -1;
    const JitRun &r = runs[k];
    const DInstr &last = P.code[r.pc + r.len - 1];
    const uint32_t tgt = last.w3, cpc = r.pc + r.len - 1;
    if (op_of(last) != OP_CALL || cost || !inl_env || !start.count(tgt)) return;
    const JitRun &rf = runs[start[tgt]];
    const uint32_t L = last.w1 & 0xFFFFu, fb = P.global_cells;
    const uint32_t off = L - fb;
    auto nx = fentry.upper_bound(tgt);
    const uint32_t fend = nx == fentry.end() ? uint32_t(P.code.size()) : nx->first;
    // (a call enters past its callee's ZERO_LOCALS: the call zeroes the locals itself)
    bool ok = op_of(P.code[rf.pc + rf.len - 1]) == OP_RET && rf.pc + rf.len == fend &&
              func_of(tgt) >= 0 && L >= fb && off % 2 == 0 && off < 255 &&
              uint64_t(P.total_cells()) + off <= TC_VF_CELLS;
    for (uint32_t i = 0; ok && i + 1 < rf.len; i++) {
      const uint16_t o = op_of(P.code[rf.pc + i]);
      ok = !ends_run(o) && o != OP_POST_CALL;
    }
    auto pm = start.find(cpc + 1);
    ok = ok && pm != start.end() && op_of(P.code[cpc + 1]) == OP_POST_CALL &&
         (P.code[cpc + 1].w1 & 0xFFFFu) == L;
    if (ok) { *inl_f = int64_t(start[tgt]); *inl_post = int64_t(pm->second); }
  };
  // runs compiled twice more for loop-carried forwarding (FwdPlan): (k, 0) every run,
  // (R, 1) the copy entered with F valid, (Pp, 2) the post-call copy that enters it
  const char *fwe = getenv("WB_FWD");   // 0: no forwarding copies (A/B aid)
  const bool fwd_store = !(getenv("WB_FWD_STORE") && getenv("WB_FWD_STORE")[0] == '0');
  const bool fwd_alias = !(getenv("WB_FWD_ALIAS") && getenv("WB_FWD_ALIAS")[0] == '0');
  std::map<size_t, FwdPlan> plans;      // R -> plan
  std::map<size_t, size_t> loop_of;     // Pp -> R
  std::vector<std::pair<size_t, int>> jobs;
  for (size_t k = 0; k < runs.size(); k++) jobs.push_back({k, 0});
  for (size_t k = 0; k < runs.size() && !(fwe && fwe[0] == '0'); k++) {
    int64_t f, post;
    inline_of(k, &f, &post);
    FwdPlan pl;
    if (f < 0 || loop_of.count(size_t(post)) || size_t(post) == k ||
        !fwd_plan(P, runs, k, size_t(f), size_t(post), &pl))
      continue;
    plans[k] = pl;
    loop_of[size_t(post)] = k;
    jobs.push_back({k, 1});
    jobs.push_back({size_t(post), 2});
  }
  // runs an inlined call returns into (past their POST_CALL: Lpa) never read their RET
  // record along with the POST_CALL (Em::ret_pf), which that path skips
  std::vector<uint8_t> inl_target(runs.size(), 0);
  for (size_t k = 0; k < runs.size(); k++) {
    int64_t f, post;
    inline_of(k, &f, &post);
    if (post >= 0) inl_target[size_t(post)] = 1;
  }
  const bool ret_pf_on = !(getenv("WB_RET_PF") && getenv("WB_RET_PF")[0] == '0');
  for (size_t jb = 0; jb < jobs.size(); jb++) {
    const size_t k = jobs[jb].first;
    const int var = jobs[jb].second;
    const JitRun &r = runs[k];
    Em e;
    e.ret_pf = ret_pf_on && !cost && !inl_target[k] && ret_prefetch_run(P, r);
    e.g = glog;
    e.run = uint32_t(k + size_t(var) * 2 * runs.size());   // (stub labels apart)
    const std::string K = std::to_string(k) + (var == 1 ? "c" : var == 2 ? "p" : "");
    if (!nob.empty()) e.nanobs = &nob;
    e.l(".p2align 6");
    e.l("Lb%s:", K.c_str());
    const DInstr &last = P.code[r.pc + r.len - 1];
    const uint16_t lop = op_of(last);
    // Where the run goes on: the instruction after it (fall-through, untaken branch), a
    // call's or branch's target, or (return) the popped return pc. The instruction after
    // the run is prefetched into both banks while the run works, unless it starts a
    // compiled run itself (then the code jumps there) or the run calls.
    const uint32_t fall = r.pc + r.len;
    const uint32_t tgt = (lop == OP_CALL || lop == OP_TAIL_CALL || is_branch_op(lop)) ? last.w3 : 0;
    const uint32_t pre = lop == OP_CALL || lop == OP_TAIL_CALL ? tgt : fall;
    const bool preload = lop != OP_RET && lop != OP_JMP && lop != OP_BR_TABLE && !start.count(pre);
    e.fb = P.global_cells;
    e.prog = &P;
    if (preload) {
      e.l("s_waitcnt lgkmcnt(0)");
      e.l("s_mov_b32 s68, 0x%x", pre * 32u);
      e.l("s_load_dwordx8 s[76:83], s[60:61], s68");
      e.l("s_load_dwordx8 s[84:91], s[60:61], s68 offset:0x20");
    }
    // metered: the price of each way out, and the entry check against the dearest
    uint64_t c_fall = 0;
    int64_t c_adj = 0;
    if (cost) {
      e.metered = true;
      for (uint32_t i = 0; i < r.len; i++) c_fall += cost->full(P, r.pc + i);
      if (is_branch_op(lop)) c_adj = cost->taken(tgt, int32_t(int16_t(last.w2 >> 16)));
      const uint64_t c_max = c_adj > 0 ? c_fall + uint64_t(c_adj) : c_fall;
      e.pc = r.pc;
      e.l("s_mov_b32 s68, 0x%x", uint32_t(c_max));
      e.l("s_mov_b32 s69, 0x%x", uint32_t(c_max >> 32));
      e.l("v_lshl_add_u64 %s, v[96:97], 0, s[68:69]", XP);
      e.l("v_cmp_gt_u64_e64 %s, %s, v[94:95]", T2, XP);   // past the limit
      e.l("v_cmp_lt_u64_e32 vcc, %s, v[96:97]", XP);      // or wrapped
      e.l("s_or_b64 %s, %s, vcc", T2, T2);
      e.leave_if_t2();
    }
    // POST_CALL ... CALL: one call-stack check at the start for both (the POST_CALL pops
    // `pop` slots, the CALL pushes n + 1), leaving before the run when either would.
    // Not where an inlined call enters past the POST_CALL (Lpa), nor for an inlined CALL.
    {
      int64_t f0 = -1, p0 = -1;
      inline_of(k, &f0, &p0);
      const DInstr &first = P.code[r.pc];
      const uint32_t fbc = P.global_cells;
      if (!inl_target[k] && f0 < 0 && lop == OP_CALL && r.len >= 2 &&
          op_of(first) == OP_POST_CALL && (first.w1 & 0xFFFFu) >= fbc &&
          (last.w1 & 0xFFFFu) >= fbc) {
        const uint32_t pop = (first.w1 & 0xFFFFu) - fbc, push = (last.w1 & 0xFFFFu) - fbc + 1;
        e.pc = r.pc;
        if (push > pop) {
          e.l("v_add_u32_e32 %s, %u, v102", X0, push - pop);
          e.l("v_cmp_lt_u32_e64 %s, s93, %s", T2, X0);
        } else {
          e.l("v_cmp_lt_u32_e64 %s, s93, v102", T2);
        }
        e.leave_if_t2();
        e.call_checked = true;
      }
    }
    std::string extra;   // SIMT split code, placed after the run
    std::vector<int> lead;
    const std::vector<MemGroup> groups = jit_groups(P, r, &lead);
    const size_t body_at = e.o.size();
    const std::string xs = "Lxs" + K;
    const uint32_t nbody = ends_run(lop) ? r.len - 1 : r.len;
    const std::vector<LoadBatch> batches = batching ? load_batches(P, r, nbody, lead)
                                                    : std::vector<LoadBatch>();
    size_t nb = 0;
    const FoldPlan fp = plan_folds(P, r, nbody, live, nob, batches);
    // an any_true that only feeds the run's br_if / br_unless (its cell dead where the run
    // goes on): the branch tests the OR of the vector's words itself (SIMT: a split stays in
    // the compiled code, so nothing outside reads the cell)
    uint32_t fuse_cell = ~0u;
    if ((sx & 1) && !cost && nbody >= 1 && nbody < r.len && !live.empty() &&
        (lop == OP_BR_IF || lop == OP_BR_UNLESS) && !fp.skip[nbody - 1]) {
      const DInstr &A = P.code[r.pc + nbody - 1];
      const uint32_t C = A.w2 & 0xFFFFu;
      bool inb = false;
      for (const auto &b : batches) inb = inb || (b.i0 <= nbody - 1 && nbody - 1 < b.i1);
      auto lv = [&](uint32_t pc) { return pc >= live.size() || (live[pc][C >> 6] >> (C & 63) & 1); };
      if (op_of(A) == OP_V_ANY_TRUE && (last.w1 & 0xFFFFu) == C && !inb &&
          !lv(r.pc + r.len) && !lv(last.w3))
        fuse_cell = C;
    }
    // ... and the f64x2 compare right before it whose mask it reads: the branch takes the
    // compare's lane masks (WB_FOLD=0 turns this off with the rest)
    bool cmp_any = false;
    if (fuse_cell != ~0u && nbody >= 2 && !fp.skip[nbody - 2] && cmp_any_on) {
      const DInstr &Cm = P.code[r.pc + nbody - 2], &A = P.code[r.pc + nbody - 1];
      const uint16_t co = op_of(Cm);
      bool inb = false;
      for (const auto &b : batches) inb = inb || (b.i0 <= nbody - 2 && nbody - 2 < b.i1);
      cmp_any = co >= OP_V_F64X2_EQ && co <= OP_V_F64X2_GE && (Cm.w2 & 0xFFFFu) == (A.w1 & 0xFFFFu) && !inb;
    }
    for (uint32_t i = 0; i < nbody; i++) {
      if (nb < batches.size() && batches[nb].i0 == i) {
        const LoadBatch &b = batches[nb++];
        emit_batch(e, P, r.pc, b, groups, lead);
        for (uint32_t k = b.i0; k < b.i1; k++) {
          e.done += (P.code[r.pc + k].w0 >> 16) & 0xFFu;
          if (cost) e.cdone += cost->full(P, r.pc + k);
        }
        i = b.i1 - 1;
        continue;
      }
      const DInstr &I = P.code[r.pc + i];
      if (fp.skip[i]) {   // a folded constant: counted, never materialized
        e.done += (I.w0 >> 16) & 0xFFu;
        if (cost) e.cdone += cost->full(P, r.pc + i);
        continue;
      }
      e.pc = r.pc + i;
      e.group = lead[i] >= 0 ? &groups[size_t(lead[i])] : nullptr;
      auto fit = fp.at.find(i);
      if (fit != fp.at.end())
        for (const auto &kv : fit->second) e.kfold[kv.first] = kv.second;
      e.fuse_any = fuse_cell != ~0u && i + 1 == nbody;
      e.cmp_any = cmp_any && i + 2 >= nbody;
      const bool ok_emit = emit(e, I);
      e.kfold.clear();
      e.fuse_any = false;
      e.cmp_any = false;
      if (!ok_emit) return "";   // jit_runs only picks compilable instructions
      e.done += (I.w0 >> 16) & 0xFFu;
      if (cost) e.cdone += cost->full(P, r.pc + i);
      // an inlined call goes on here, after the POST_CALL it makes unnecessary
      if (i == 0 && op_of(I) == OP_POST_CALL) e.l("Lpa%s:", K.c_str());
    }
    e.drain();
    if (sched) e.o = e.o.substr(0, body_at) + schedule(e.o.substr(body_at));
    e.pc = r.pc + r.len - 1;
    e.group = nullptr;
    // go to pc `to` (PCOFF and CNT set): straight into its compiled run when it has one
    // (in diverged mode only if that run stops short of the lowest waiting pc, as the
    // JIT slot would check), else through its TInstr (banks: already loaded for it)
    int lab = 0;
    auto go = [&](uint32_t to, bool banks) {
      auto it = start.find(to);
      const std::string disp = "Ld" + K + "_" + std::to_string(lab++);
      if (it != start.end()) {
        e.l("s_add_u32 s68, s62, 0x%x", (runs[it->second].len - 1) * 32u);
        e.l("s_cmp_ge_u32 s68, s63");
        e.l("s_cbranch_scc1 %s", disp.c_str());
        // (a long jump: the code object can outgrow s_branch's +-128 KiB); a forwarding
        // loop's post-call copy enters its run's forwarding copy
        const std::string q = "Lq" + K + "_" + std::to_string(lab);
        const std::string tl = "Lb" + std::to_string(it->second) +
                               (var == 2 && loop_of.count(k) && loop_of[k] == it->second ? "c" : "");
        long_jump(e, tl, q);
        e.l("%s:", disp.c_str());
        banks = false;
      }
      e.l("s_waitcnt lgkmcnt(0)");
      if (!banks) {
        e.l("s_load_dwordx8 s[76:83], s[60:61], s62");
        e.l("s_load_dwordx8 s[84:91], s[60:61], s62 offset:0x20");
        e.l("s_waitcnt lgkmcnt(0)");
      }
      e.l("s_add_u32 s68, s70, s76");
      e.l("s_addc_u32 s69, s71, 0");
      e.l("s_setpc_b64 s[68:69]");
    };
    // a taken transfer: the core's taken() checks (count limit; diverged: a jump to or
    // below the lowest waiting pc re-aims OTHER, reaching OTHER goes to the scheduler)
    auto taken_checks = [&]() {
      e.l("s_cmp_ge_u32 s65, s64");
      e.l("s_cbranch_scc1 %s", xs.c_str());
      e.l("s_cmp_le_u32 s62, s95");
      e.l("s_cselect_b32 s63, s95, s63");
      e.l("s_cmp_ge_u32 s62, s63");
      e.l("s_cbranch_scc1 %s", xs.c_str());
    };
    // The common case of a transfer to pc `to` that starts a compiled run, in one branch:
    // (taken) the count limit is not reached, and after the re-aim that run stops short of
    // OTHER -- the jump goes straight there; else the full checks below (go, taken_checks)
    // run as before. `lim`: the limit is already in s68 (budget ? OTHER : 0) -- a return's
    // shared prefix, see below.
    int nfast = 0;
    auto fast_to = [&](uint32_t to, bool taken, bool lim) {
      auto it = start.find(to);
      if (it == start.end()) return;
      const uint32_t tend = (to + runs[it->second].len - 1) * 32u;
      const std::string tl = "Lb" + std::to_string(it->second) +
                             (var == 2 && loop_of.count(k) && loop_of[k] == it->second ? "c" : "");
      if (lim) {
        e.l("s_cmp_gt_u32 s68, 0x%x", tend);
      } else if (taken) {
        if (to == 0) {   // (pc 0 <= LOW always)
          e.l("s_mov_b32 s63, s95");
        } else {
          e.l("s_cmp_ge_u32 s95, 0x%x", to * 32u);   // to <= LOW: re-aim OTHER
          e.l("s_cselect_b32 s63, s95, s63");
        }
        e.l("s_cmp_lt_u32 s65, s64");
        e.l("s_cselect_b32 s68, s63, 0");
        e.l("s_cmp_gt_u32 s68, 0x%x", tend);
      } else {
        e.l("s_cmp_gt_u32 s63, 0x%x", tend);
      }
      cond_jump(e, tl, "Lf" + K + "_" + std::to_string(nfast++));
    };
    auto fallthrough = [&](uint32_t cnt) {   // next(): stop at the lowest waiting pc
      e.gas_add(c_fall);
      e.l("s_add_u32 s65, s65, 0x%x", cnt);
      fast_to(fall, false, false);
      e.l("s_mov_b32 s62, 0x%x", fall * 32u);
      e.l("s_cmp_ge_u32 s62, s63");
      e.l("s_cbranch_scc1 %s", xs.c_str());
      go(fall, preload);
    };
    int64_t inl_f = -1, inl_post = -1;
    inline_of(k, &inl_f, &inl_post);
    const FwdPlan *fwd = plans.count(k) ? &plans[k] : nullptr;
    if (inl_f >= 0) {
      const JitRun &rf = runs[size_t(inl_f)];
      const uint32_t L = last.w1 & 0xFFFFu, nargs = last.w1 >> 16, nloc = last.w2 & 0xFFFFu;
      const uint32_t fb = P.global_cells, off = L - fb, n = L - fb, callpc = e.pc;
      const std::string IK = "i" + K;
      // the real call's LDS check first: a call that would pass the LDS part of the call
      // stack leaves before the CALL (the C++ step makes it), as without inlining
      e.l("v_add_u32_e32 %s, %u, v102", X0, n + 1);
      e.l("v_cmp_lt_u32_e64 %s, s93, %s", T2, X0);
      e.leave_if_t2();
      const std::vector<uint8_t> dead = dead_zeros(P, rf);
      Em ei;
      ei.g = glog;
      ei.run = e.run + uint32_t(runs.size());   // (labels apart from every real run's)
      ei.fb = fb;
      ei.prog = &P;
      ei.shift = off;
      ei.nanobs = e.nanobs;
      ei.done = r.cnt;                      // counted before the callee: the caller's run
      for (uint32_t q = 0; q < nloc; q++)
        if (dead.empty() || !dead[fb + nargs + q]) ei.l("v_mov_b32 %s, 0", ei.v(fb + nargs + q));
      std::vector<int> lead2;
      const std::vector<MemGroup> groups2 = jit_groups(P, rf, &lead2);
      const size_t body2 = ei.o.size();
      const bool fc = fwd && var == 1;   // the forwarding copy: the callee's loads from F
      int64_t renamed = -1;              // the stack cell computed into a word's VGPR
      std::vector<std::pair<uint32_t, uint32_t>> deferred;   // (cell, VGPR) read, then written
      const std::vector<LoadBatch> batches2 = batching && !fc ? load_batches(P, rf, rf.len - 1, lead2)
                                                              : std::vector<LoadBatch>();
      size_t nb2 = 0;
      for (uint32_t i = 0; i + 1 < rf.len; i++) {
        if (nb2 < batches2.size() && batches2[nb2].i0 == i) {
          const LoadBatch &b = batches2[nb2++];
          emit_batch(ei, P, rf.pc, b, groups2, lead2);
          for (uint32_t k = b.i0; k < b.i1; k++) {
            ei.done += (P.code[rf.pc + k].w0 >> 16) & 0xFFu;
            if (fwd && fwd->copy_now[k]) {
              const uint32_t c = P.code[rf.pc + k].w2 & 0xFFFFu;
              ei.sync({c});
              ei.l("v_mov_b32 v%u, %s", fwd->freg.at(uint32_t(fwd->addr[k])), ei.v(c));
            }
          }
          i = b.i1 - 1;
          continue;
        }
        const DInstr &I = P.code[rf.pc + i];
        ei.pc = rf.pc + i;
        ei.group = lead2[i] >= 0 ? &groups2[size_t(lead2[i])] : nullptr;
        const int64_t fa = fwd ? fwd->addr[i] : -1;
        if (fa >= 0 && fc && op_of(I) == OP_LD32) {
          // (a group that also stores still computes its base: its stores use it)
          if (ei.group && ei.group->store_end) group_base(ei, *ei.group);
          ei.group = nullptr;
          const uint32_t c = I.w2 & 0xFFFFu;
          ei.sync({c});
          if (fwd_alias) ei.amap[c] = fwd->freg.at(uint32_t(fa));
          else ei.l("v_mov_b32 %s, v%u", ei.v(c), fwd->freg.at(uint32_t(fa)));
          ei.done += (I.w0 >> 16) & 0xFFu;
          continue;
        }
        if (!ei.amap.empty() && !(fa >= 0 && op_of(I) == OP_ST32 && fwd_store)) {
          // an aliased cell this instruction writes gets its own register back first if
          // the instruction also reads it (else the alias just ends); anything but a plain
          // 32-bit op (which might leave, or names register pairs) gets every cell back
          std::vector<uint32_t> w;
          const bool ex = written_exact(I, &w);
          std::vector<uint32_t> cells;
          for (const auto &kv : ei.amap) cells.push_back(kv.first);
          for (uint32_t x : cells) {
            const bool wr = std::find(w.begin(), w.end(), x) != w.end();
            const bool rd = (I.w1 & 0xFFFFu) == x || (I.w1 >> 16) == x || (I.w2 >> 16) == x ||
                            (op_of(I) == OP_I32_ADD3_XROTR_I && (I.w3 & 0xFFFFu) == x);
            size_t shared = 0;
            for (const auto &kv : ei.amap) shared += kv.second == ei.amap[x];
            if (ex && wr && rd && shared == 1) deferred.push_back({x, ei.amap[x]});
            else if (!ex || (wr && rd)) ei.materialize(x);
            else if (wr) ei.amap.erase(x);
          }
        }
        if (fa >= 0 && op_of(I) == OP_ST32 && fwd_store) {
          // the word goes to its VGPR first and is stored from there: the stack cell that
          // held it is free at once for the next value (no wait for the store's data read)
          const std::string fr = "v" + std::to_string(fwd->freg.at(uint32_t(fa)));
          ei.before_write(fwd->freg.at(uint32_t(fa)));
          if (renamed != int64_t(I.w1 >> 16)) {
            ei.sync({I.w1 >> 16});
            ei.l("v_mov_b32 %s, %s", fr.c_str(), ei.v(I.w1 >> 16));
          }
          renamed = -1;
          if (fc) {   // (the first trip checked these constant addresses, raised the mark)
            if (ei.group) group_base(ei, *ei.group);
            ei.group = nullptr;
          }
          emit_store(ei, OP_ST32, I.w1 & 0xFFFFu, I.w1 >> 16, I.w3, fr.c_str());
          ei.done += (I.w0 >> 16) & 0xFFu;
          continue;
        }
        // a stack cell computed only to be stored as a forwarded word (it is dead after
        // the store pops it): computed straight into the word's VGPR
        renamed = -1;
        // (only in the copy: there the store cannot leave, which would need the cell)
        if (fc && fwd_store && i + 2 < rf.len && fwd->addr[i + 1] >= 0 &&
            op_of(P.code[rf.pc + i + 1]) == OP_ST32) {
          const uint32_t y = P.code[rf.pc + i + 1].w1 >> 16;
          std::vector<uint32_t> w;
          written_exact(I, &w);
          const bool srcs = (I.w1 & 0xFFFFu) != y && (I.w1 >> 16) != y && (I.w2 >> 16) != y &&
                            (op_of(I) != OP_I32_ADD3_XROTR_I || (I.w3 & 0xFFFFu) != y);
          if (y >= fb + nargs + nloc && w.size() == 1 && w[0] == y && srcs &&
              op_of(I) != OP_LD32 && !mem_bytes(op_of(I))) {
            ei.sync({y});
            ei.before_write(fwd->freg.at(uint32_t(fwd->addr[i + 1])));
            ei.alias_cell = y;
            ei.alias_reg = fwd->freg.at(uint32_t(fwd->addr[i + 1]));
            renamed = y;
          }
        }
        const size_t mark = ei.o.size();
        if (!emit(ei, I)) return "";
        ei.alias_cell = -1;
        // A cell read through its alias and written by this instruction: the instruction
        // read the word's VGPR; its first line that writes the VGPR writes the cell's own
        // register instead, and later lines read that (else: the cell back first, again)
        for (const auto &dx : deferred) {
          const std::string fv = "v" + std::to_string(dx.second);
          const std::string rv = "v" + std::to_string(128 + ei.sc(dx.first));
          std::string out;
          bool written = false;
          for (size_t at = mark; at < ei.o.size();) {
            size_t nl = ei.o.find('\n', at);
            std::string ln = ei.o.substr(at, nl - at);
            at = nl + 1;
            const size_t sp = ln.find(' ');
            if (!written && ln.compare(0, 2, "v_") == 0 && sp != std::string::npos &&
                ln.compare(sp + 1, fv.size(), fv) == 0 &&
                (sp + 1 + fv.size() == ln.size() || ln[sp + 1 + fv.size()] == ',')) {
              ln = ln.substr(0, sp + 1) + rv + ln.substr(sp + 1 + fv.size());
              written = true;
            } else if (written) {
              for (size_t q = ln.find(fv); q != std::string::npos; q = ln.find(fv, q + rv.size())) {
                const size_t e2 = q + fv.size();
                if ((q == 0 || !isalnum((unsigned char)ln[q - 1])) &&
                    (e2 == ln.size() || !isdigit((unsigned char)ln[e2])))
                  ln = ln.substr(0, q) + rv + ln.substr(e2);
              }
            }
            out += ln + "\n";
          }
          if (written) {
            ei.o = ei.o.substr(0, mark) + out;
            ei.amap.erase(dx.first);
          } else {   // (not expected: every exact write names the cell's register)
            ei.o.resize(mark);
            ei.materialize(dx.first);
            if (!emit(ei, I)) return "";
          }
        }
        deferred.clear();
        if (fa >= 0 && op_of(I) == OP_ST32) {   // (WB_FWD_STORE=0: copied after the store)
          ei.before_write(fwd->freg.at(uint32_t(fa)));
          ei.l("v_mov_b32 v%u, %s", fwd->freg.at(uint32_t(fa)), ei.v(I.w1 >> 16));
        }
        if (fa >= 0 && fwd->copy_now[i]) {
          ei.sync({I.w2 & 0xFFFFu});
          ei.l("v_mov_b32 v%u, %s", fwd->freg.at(uint32_t(fa)), ei.v(I.w2 & 0xFFFFu));
        }
        ei.done += (I.w0 >> 16) & 0xFFu;
      }
      ei.drain();
      if (fwd && !fc)
        for (const auto &fc2 : fwd->end_copy) ei.l("v_mov_b32 v%u, v%u", fc2.first, 128 + fc2.second);
      ei.group = nullptr;
      if (sched) ei.o = ei.o.substr(0, body2) + schedule(ei.o.substr(body2));
      // the return: results (shifted cells a..) to L.., every instruction counted, on after
      // the caller's POST_CALL (its run's banks as that run would have loaded them)
      const DInstr &rt = P.code[rf.pc + rf.len - 1];
      const uint32_t ra = rt.w1 & 0xFFFFu, nres = rt.w1 >> 16;
      for (uint32_t q = 0; q < nres; q++)
        ei.l("v_mov_b32 v%u, %s", 128 + L + q, ei.v(ra + q));
      ei.amap.clear();   // (the callee's cells are dead once its results are out)
      ei.l("s_add_u32 s65, s65, 0x%x", r.cnt + rf.cnt);
      {
        const JitRun &rp = runs[size_t(inl_post)];
        const DInstr &pl = P.code[rp.pc + rp.len - 1];
        const uint16_t plo = op_of(pl);
        const uint32_t ptgt = (plo == OP_CALL || is_branch_op(plo)) ? pl.w3 : 0;
        const uint32_t ppre = plo == OP_CALL ? ptgt : rp.pc + rp.len;
        if (plo != OP_RET && plo != OP_JMP && plo != OP_BR_TABLE && !start.count(ppre)) {
          ei.l("s_waitcnt lgkmcnt(0)");
          ei.l("s_mov_b32 s68, 0x%x", ppre * 32u);
          ei.l("s_load_dwordx8 s[76:83], s[60:61], s68");
          ei.l("s_load_dwordx8 s[84:91], s[60:61], s68 offset:0x20");
        }
      }
      ei.l("s_mov_b32 s62, 0x%x", (callpc + 1) * 32u);
      long_jump(ei, "Lpa" + std::to_string(inl_post) + (fwd ? "p" : ""), "Lpq" + IK);
      // leaves inside the callee: make the call real first
      std::string deopt;
      {
        Em d;
        d.l("s_waitcnt vmcnt(0)");   // (the callee's loads in flight land before the moves)
        d.l("v_lshl_add_u32 %s, v102, 8, v103", X1);
        for (uint32_t q = 0; q < n; q++) d.l("ds_write_b32 %s, v%u offset:%u", X1, 128 + fb + q, q * 256u);
        d.l("v_mov_b32 %s, 0x%x", Y1, ((callpc + 1) & 0xFFFFFu) | (L << 20));
        d.l("ds_write_b32 %s, %s offset:%u", X1, Y1, n * 256u);
        d.l("v_add_u32_e32 v102, %u, v102", n + 1);
        for (uint32_t c = fb; c < P.total_cells(); c++) d.l("v_mov_b32 v%u, v%u", 128 + c, 128 + c + off);
        deopt = d.o;
      }
      ei.o += ei.tail;
      for (const auto &st : ei.stubs) {
        ei.o += st.lab + ":\n" + deopt;
        ei.l("s_mov_b32 s62, 0x%x", st.pc * 32u);
        ei.l("s_add_u32 s65, s65, 0x%x", st.done);
        ei.l("s_setpc_b64 s[70:71]");
      }
      // the callee's code follows the caller's (falls through into it; its block counts
      // the caller's run)
      e.l("Li%s:", IK.c_str());
      e.o += ei.o;
    } else if (lop == OP_TAIL_CALL) {
      std::vector<uint8_t> dead;
      if (start.count(tgt)) dead = dead_zeros(P, runs[start[tgt]]);
      emit_tail_call(e, last, dead.empty() ? nullptr : &dead);
      e.gas_add(c_fall);
      e.l("s_add_u32 s65, s65, 0x%x", r.cnt);
      fast_to(tgt, true, false);
      e.l("s_mov_b32 s62, 0x%x", tgt * 32u);
      taken_checks();
      go(tgt, preload);
    } else if (lop == OP_CALL) {
      std::vector<uint8_t> dead;
      if (start.count(tgt)) dead = dead_zeros(P, runs[start[tgt]]);
      emit_call(e, last, e.pc, dead.empty() ? nullptr : &dead);
      e.gas_add(c_fall);
      e.l("s_add_u32 s65, s65, 0x%x", r.cnt);
      fast_to(tgt, true, false);
      e.l("s_mov_b32 s62, 0x%x", tgt * 32u);
      taken_checks();
      go(tgt, preload);
    } else if (lop == OP_RET) {
      // a return's likely targets: the instruction after each direct call of its function
      std::vector<uint32_t> sites;
      const int64_t f = func_of(e.pc);
      if (f >= 0)
        for (uint32_t rs : ret_sites[uint32_t(f)])
          if (start.count(rs) && sites.size() < 6) sites.push_back(rs);
      // the first two sites' return records are constants: a group whose lanes all hold one
      // of them goes straight to Lrk<K>_<q> (below)
      std::vector<std::pair<uint32_t, std::string>> known;
      for (size_t q = 0; q < sites.size() && q < 2 && !cost; q++) {
        const DInstr &cl = P.code[sites[q] - 1];
        const uint32_t L = cl.w1 & 0xFFFFu;
        if (op_of(cl) == OP_CALL && L < 4096)
          known.push_back({(sites[q] & 0xFFFFFu) | (L << 20), "Lrk" + K + "_" + std::to_string(q)});
      }
      const std::string rout = emit_ret(e, last, (sx & 2) ? "Lrs" + K : std::string(), known);
      if (sx & 2) {
        // lanes returning to different places: each records its return pc and count
        // (unless one leaves the entry function: the C++ step finishes those) and the
        // scheduler picks who goes on
        const uint32_t a = last.w1 & 0xFFFFu, nres = last.w1 >> 16, fb = e.fb;
        Em x;
        x.l("Lrs%s:", K.c_str());
        x.l("v_and_b32_e32 %s, 0xfffff, %s", X0, Y1);
        x.l("v_cmp_eq_u32_e32 vcc, 0xfffff, %s", X0);
        x.l("s_and_b64 vcc, vcc, exec");
        x.l("s_cbranch_vccnz %s", rout.c_str());
        x.l("v_subrev_u32_e32 v102, 1, v102");
        for (uint32_t q = 0; q < nres; q++)
          if (a != fb) x.l("v_mov_b32 %s, %s", x.V(fb + q).c_str(), x.V(a + q).c_str());
        x.l("v_mov_b32 %s, %s", VPC, X0);
        x.l("s_add_u32 s65, s65, 0x%x", r.cnt);
        flush(x);
        long_jump(x, "Lsched", "Lrq" + K);
        extra += x.o;
      }
      e.gas_add(c_fall);
      e.l("s_add_u32 s65, s65, 0x%x", r.cnt);
      // straight into the code after a known call site of this function, else dispatch
      // the fast way: re-aim, s68 = the limit (budget ? OTHER : 0), then per known site
      // one compare against the site's run end (fast_to)
      if (!sites.empty()) {
        e.l("s_cmp_le_u32 s62, s95");
        e.l("s_cselect_b32 s63, s95, s63");
        e.l("s_cmp_lt_u32 s65, s64");
        e.l("s_cselect_b32 s68, s63, 0");
        // the limit clears every site's run (converged: always): straight to the site
        uint32_t maxend = 0;
        std::vector<std::string> tls;
        for (uint32_t rs : sites) {
          const size_t ri = start[rs];
          maxend = std::max(maxend, (rs + runs[ri].len - 1) * 32u);
          tls.push_back("Lb" + std::to_string(ri) + (var == 2 && loop_of.count(k) && loop_of[k] == ri ? "c" : ""));
        }
        e.l("s_cmp_gt_u32 s68, 0x%x", maxend);
        e.l("s_cbranch_scc0 Lrg%s", K.c_str());
        for (size_t q = 0; q < sites.size(); q++) {
          e.l("s_cmp_eq_u32 s62, 0x%x", sites[q] * 32u);
          cond_jump(e, tls[q], "Lrj" + K + "_" + std::to_string(q));
        }
        e.l("Lrg%s:", K.c_str());
        for (size_t q = 0; q < sites.size(); q++) {
          e.l("s_cmp_eq_u32 s62, 0x%x", sites[q] * 32u);
          e.l("s_cbranch_scc1 Lrf%s_%zu", K.c_str(), q);
        }
      }
      taken_checks();
      for (size_t q = 0; q < sites.size(); q++) {
        e.l("s_cmp_eq_u32 s62, 0x%x", sites[q] * 32u);
        e.l("s_cbranch_scc1 Lrt%s_%zu", K.c_str(), q);
      }
      go(~0u, false);
      for (size_t q = 0; q < sites.size(); q++) {
        e.l("Lrf%s_%zu:", K.c_str(), q);
        fast_to(sites[q], true, true);
        taken_checks();
        e.l("Lrt%s_%zu:", K.c_str(), q);
        go(sites[q], false);
      }
      // every lane returns to known site q: pop, results, then the transfer's checks
      for (size_t q = 0; q < known.size(); q++) {
        const uint32_t a = last.w1 & 0xFFFFu, nres = last.w1 >> 16, fb = e.fb;
        e.l("%s:", known[q].second.c_str());
        e.l("v_subrev_u32_e32 v102, 1, v102");
        for (uint32_t c = 0; c < nres; c++)
          if (a != fb) e.l("v_mov_b32 %s, %s", e.V(fb + c).c_str(), e.V(a + c).c_str());
        e.l("s_add_u32 s65, s65, 0x%x", r.cnt);
        fast_to(sites[q], true, false);
        e.l("s_mov_b32 s62, 0x%x", sites[q] * 32u);
        taken_checks();
        go(sites[q], false);
      }
    } else if (lop == OP_BR_TABLE) {
      emit_br_table(e, last);
      // every lane to the same entry: jump there (count + that entry's correction);
      // else (SIMT) each lane records its target and count and the scheduler picks, or
      // (no SIMT) the C++ step splits the wave
      e.l("v_readfirstlane_b32 s68, %s", Y0);
      e.l("v_readfirstlane_b32 s69, %s", Y1);
      e.l("s_nop 1");
      e.l("v_cmp_ne_u32_e64 %s, s68, %s", T2, Y0);
      e.l("v_cmp_ne_u32_e32 vcc, s69, %s", Y1);
      e.l("s_or_b64 %s, %s, vcc", T2, T2);
      e.l("s_and_b64 %s, %s, exec", T2, T2);
      if (sx & 1) {
        e.l("s_cbranch_scc1 Lts%s", K.c_str());
        Em x;
        x.l("Lts%s:", K.c_str());
        x.l("v_mov_b32 %s, %s", VPC, Y0);
        x.l("v_add_u32_e32 %s, %s, %s", VCNT, VCNT, Y1);
        x.l("s_add_u32 s65, s65, 0x%x", r.cnt);
        flush(x);
        long_jump(x, "Lsched", "Ltq" + K);
        extra += x.o;
      } else {
        const std::string lab_split = "Lx" + K + "_" + std::to_string(e.stubs.size());
        e.stubs.push_back(Em::Stub{lab_split, e.pc, e.done, e.cdone});
        e.l("s_cbranch_scc1 %s", lab_split.c_str());
      }
      e.l("s_lshl_b32 s62, s68, 5");
      e.l("s_add_u32 s65, s65, 0x%x", r.cnt);
      e.l("s_add_u32 s65, s65, s69");
      taken_checks();
      go(~0u, false);
    } else if (is_branch_op(lop)) {
      const uint32_t bcnt = (last.w0 >> 16) & 0xFFu;
      const int32_t tcnt = int32_t(int16_t(last.w2 >> 16));
      const uint32_t taken_cnt = uint32_t(int32_t(r.cnt) + tcnt);   // (cnt + tcnt >= 0)
      const std::string nt = "Lnt" + K;
      if (lop != OP_JMP) {
        if (cmp_any) {   // VCC = the lanes whose any_true is 1
          if (lop == OP_BR_UNLESS) e.l("s_not_b64 vcc, vcc");
        } else {
          if (fuse_cell != ~0u) {   // (the fused any_true's OR is in R0)
            e.alias_cell = int64_t(fuse_cell);
            e.alias_reg = 114;
          }
          branch_cond(e, last);
          e.alias_cell = -1;
        }
        e.l("s_and_b64 %s, vcc, exec", T2);
        e.l("s_cbranch_scc0 %s", nt.c_str());    // no lane takes it
        e.l("s_cmp_eq_u64 %s, exec", T2);
        if (sx & 1) {
          // lanes disagree: each records where it goes on (vcc: taken) and its count,
          // and the scheduler picks who goes first
          e.l("s_cbranch_scc0 Lbs%s", K.c_str());
          Em x;
          x.l("Lbs%s:", K.c_str());
          {   // (inline constants where they fit: VOP3 selects take -16..64)
            auto inl = [](int64_t v) { return v >= -16 && v <= 64; };
            std::string f = std::to_string(fall), t = std::to_string(tgt);
            if (!inl(fall)) { x.l("v_mov_b32 %s, 0x%x", X0, fall); f = X0; }
            if (!inl(tgt)) { x.l("v_mov_b32 %s, 0x%x", X1, tgt); t = X1; }
            x.l("v_cndmask_b32_e64 %s, %s, %s, vcc", VPC, f.c_str(), t.c_str());
            if (inl(tcnt)) {   // a taken branch's correction
              x.l("v_cndmask_b32_e64 %s, 0, %d, vcc", X0, int32_t(tcnt));
            } else {
              x.l("v_mov_b32 %s, 0x%x", X1, uint32_t(tcnt));
              x.l("v_cndmask_b32_e32 %s, 0, %s, vcc", X0, X1);
            }
            x.l("v_add_u32_e32 %s, %s, %s", VCNT, VCNT, X0);
          }
          x.l("s_add_u32 s65, s65, 0x%x", r.cnt);
          flush(x);
          if (fall != tgt && !hybrid && !depth_pick) {   // (hybrid: every split goes to Lsched, hence the trips)
            // No waiting lane at or below the nearer destination `lo`: the lanes going
            // there are the next group, those going to `hi` wait, and the lowest waiting
            // pc becomes min(LOW, hi) -- a pick without the wave reductions of Lsched
            const uint32_t lo = std::min(fall, tgt), hi = std::max(fall, tgt);
            x.l("s_cmp_le_u32 s95, 0x%x", lo * 32u);
            x.l("s_cbranch_scc0 Lbf%s", K.c_str());
            long_jump(x, "Lsched", "Lbq" + K);
            x.l("Lbf%s:", K.c_str());
            x.l("s_sub_u32 s64, s64, 16");
            x.l("s_cselect_b32 s64, 0, s64");
            x.l("s_cmp_eq_u32 s95, -1");                  // converged until now: D banks
            x.l("s_cbranch_scc0 Lbm%s", K.c_str());
            x.l("s_add_u32 s70, s70, 0x%x", 2u * TC_BANK_BYTES);
            x.l("s_addc_u32 s71, s71, 0");
            x.l("s_add_u32 s72, s70, 0x%x", TC_BANK_BYTES);
            x.l("s_addc_u32 s73, s71, 0");
            x.l("Lbm%s:", K.c_str());
            x.l("s_min_u32 s95, s95, 0x%x", hi * 32u);
            x.l("s_mov_b32 s63, s95");
            x.l(lo == tgt ? "s_and_b64 s[74:75], vcc, exec" : "s_andn2_b64 s[74:75], exec, vcc");
            x.l("s_mov_b32 s62, 0x%x", lo * 32u);
            x.l("s_waitcnt lgkmcnt(0)");
            x.l("s_load_dwordx8 s[76:83], s[60:61], s62");
            x.l("s_load_dwordx8 s[84:91], s[60:61], s62 offset:0x20");
            long_jump(x, "Lsc_disp", "Lbt" + K);   // (clobbers s[68:69])
          } else {
            long_jump(x, "Lsched", "Lbq" + K);
          }
          extra += x.o;
        } else {
          const std::string lab_split = "Lx" + K + "_" + std::to_string(e.stubs.size());
          e.stubs.push_back(Em::Stub{lab_split, e.pc, e.done, e.cdone});
          e.l("s_cbranch_scc0 %s", lab_split.c_str());   // lanes disagree: the C++ step splits
        }
      }
      e.gas_add(uint64_t(int64_t(c_fall) + c_adj));
      e.l("s_add_u32 s65, s65, 0x%x", taken_cnt);
      fast_to(tgt, true, false);
      e.l("s_mov_b32 s62, 0x%x", tgt * 32u);
      taken_checks();
      go(tgt, false);
      if (lop != OP_JMP) {
        e.l("%s:", nt.c_str());
        (void)bcnt;
        fallthrough(r.cnt);
      }
    } else {
      fallthrough(r.cnt);
    }
    e.l("Lxs%s:", K.c_str());
    if (sx & 4) {   // reached a waiting lane or the count limit: merge / reschedule
      long_jump(e, "Lmerge", "Lmq" + K);
    } else {
      e.l("s_add_u32 s68, s70, %u", TC_JIT_XS);
      e.l("s_addc_u32 s69, s71, 0");
      e.l("s_setpc_b64 s[68:69]");
    }
    e.o += extra;
    e.o += e.tail;
    for (const auto &s : e.stubs) {   // leave before instruction s.pc
      e.l("%s:", s.lab.c_str());
      e.gas_add(s.cdone);
      e.l("s_mov_b32 s62, 0x%x", s.pc * 32u);
      e.l("s_add_u32 s65, s65, 0x%x", s.done);
      e.l("s_setpc_b64 s[70:71]");
    }
    body += e.o;
  }
  if (hybrid) body += trip_source(P, runs, glog, true);
  body = resolve_jumps(body);
  body += ".p2align 3\nLtab:\n";
  for (size_t k = 0; k < runs.size(); k++) body += ".quad Lb" + std::to_string(k) + " - Ltab\n";
  body += "Lend:\n";
  std::string src =
      "// generated by jit.cpp: compiled runs of the V-frame threaded core\n"
      "extern \"C\" __global__ void wbjit_addrs(unsigned long long *out, unsigned n) {\n"
      "  unsigned lo, hi;\n"
      "  asm volatile(\n";
  for (size_t at = 0; at < body.size();) {
    const size_t nl = body.find('\n', at);
    src += "      \"" + body.substr(at, nl - at) + "\\n\"\n";
    at = nl + 1;
  }
  src += "      : \"=s\"(lo), \"=s\"(hi) : : \"s6\", \"s7\", \"s8\", \"s9\", \"scc\", \"memory\");\n"
         "  const long long *tab = (const long long *)(((unsigned long long)hi << 32) | lo);\n"
         "  for (unsigned k = threadIdx.x; k < n; k += blockDim.x)\n"
         "    out[k] = (unsigned long long)tab + (unsigned long long)tab[k];\n"
         "}\n";
  return src;
}

bool trips_pay(const Program &P) {
  const size_t n = P.code.size();
  std::vector<std::pair<uint32_t, uint32_t>> spans;   // loops: (head, back-edge pc)
  auto targets = [&](size_t pc, std::vector<uint32_t> *t) {
    const DInstr &I = P.code[pc];
    const uint16_t op = op_of(I);
    t->clear();
    if (op == OP_BR_TABLE) {
      for (uint32_t k = 0; k <= (I.w1 >> 16); k++)
        if (2 * (size_t(I.w3) + k) < P.brtab.size()) t->push_back(P.brtab[2 * (size_t(I.w3) + k)]);
    } else if (is_branch_op(op) || op == OP_BR_IF_MOV1 || op == OP_BR_IF_MOV2) {
      t->push_back(I.w3);
      if (op != OP_JMP) t->push_back(uint32_t(pc + 1));
    }
  };
  std::vector<uint32_t> t;
  for (size_t pc = 0; pc < n; pc++) {
    const uint16_t op = op_of(P.code[pc]);
    if (op == OP_CALL || op == OP_CALL_INDIRECT || op == OP_TAIL_CALL || op == OP_TAIL_CALL_INDIRECT)
      return false;
    targets(pc, &t);
    for (uint32_t x : t)
      if (x <= pc) spans.push_back({x, uint32_t(pc)});
  }
  for (size_t pc = 0; pc < n; pc++) {
    targets(pc, &t);
    if (t.size() < 2) continue;
    // the innermost loop around pc
    uint32_t h = 0, e = 0, best = 0xFFFFFFFFu;
    for (const auto &sp : spans)
      if (sp.first <= pc && pc <= sp.second && sp.second - sp.first < best) {
        best = sp.second - sp.first;
        h = sp.first;
        e = sp.second;
      }
    if (best == 0xFFFFFFFFu) continue;
    std::vector<uint32_t> in;
    for (uint32_t x : t)
      if (x >= h && x <= e && std::find(in.begin(), in.end(), x) == in.end()) in.push_back(x);
    if (in.size() >= 2) return true;
  }
  return false;
}

std::string jit_compile(const std::string &src, std::vector<char> *code, const std::string &arch) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "wbjit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    return "hiprtcCreateProgram failed";
  const std::string target = "--offload-arch=" + arch;
  const char *opts[] = {target.c_str(), "-O1"};
  if (hiprtcCompileProgram(prog, 2, opts) != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n + 1, '\0');
    hiprtcGetProgramLog(prog, log.data());
    hiprtcDestroyProgram(&prog);
    return "compiled-run assembly failed: " + log.substr(0, 2000);
  }
  size_t sz = 0;
  hiprtcGetCodeSize(prog, &sz);
  code->assign(sz, 0);
  hiprtcGetCode(prog, code->data());
  hiprtcDestroyProgram(&prog);
  return "";
}

std::string jit_load(const std::string &src, size_t nruns, int device, std::vector<uint64_t> *addr) {
  // one code object per (HIP context, device, source) while that context lives: contexts
  // of the same module share it (a new primary context after hipDeviceReset gets its own)
  static std::mutex mu;
  static std::map<std::tuple<uintptr_t, int, std::string>, std::vector<uint64_t>> cache;
  std::lock_guard<std::mutex> lock(mu);
  hipCtx_t hctx = nullptr;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wdeprecated-declarations"
  (void)hipCtxGetCurrent(&hctx);
#pragma clang diagnostic pop
  const auto key = std::make_tuple(uintptr_t(hctx), device, src);
  auto it = cache.find(key);
  if (it != cache.end()) { *addr = it->second; return ""; }
  // the device's own target (gfx950 on MI355X), not a hard-coded one
  std::string arch = "gfx950";
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.gcnArchName[0]) {
    arch = prop.gcnArchName;
    const size_t colon = arch.find(':');   // (feature suffixes such as :sramecc+:xnack-)
    if (colon != std::string::npos) arch.resize(colon);
  }
  std::vector<char> code;
  std::string err = jit_compile(src, &code, arch);
  if (!err.empty()) return err;
  hipModule_t mod;
  if (hipModuleLoadData(&mod, code.data()) != hipSuccess) return "hipModuleLoadData failed";
  hipFunction_t fn;
  if (hipModuleGetFunction(&fn, mod, "wbjit_addrs") != hipSuccess) return "hipModuleGetFunction failed";
  uint64_t *dout = nullptr;
  if (hipMalloc(&dout, std::max<size_t>(1, nruns) * 8) != hipSuccess) return "hipMalloc failed";
  unsigned nr = unsigned(nruns);
  void *args[] = {&dout, &nr};
  std::vector<uint64_t> a(nruns, 0);
  // (a private stream: BatchCreate must not wait for other contexts' kernels)
  hipStream_t qs = nullptr;
  const bool ok = hipStreamCreateWithFlags(&qs, hipStreamNonBlocking) == hipSuccess &&
                  hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, qs, args, nullptr) == hipSuccess &&
                  hipMemcpyAsync(a.data(), dout, nruns * 8, hipMemcpyDeviceToHost, qs) == hipSuccess &&
                  hipStreamSynchronize(qs) == hipSuccess;
  if (qs) (void)hipStreamDestroy(qs);
  (void)hipFree(dout);
  if (!ok) return "compiled-run address query failed";
  for (uint64_t x : a)
    if (x == 0 || (x & 63)) return "compiled-run address query returned a bad address";
  cache[key] = a;   // the module stays loaded: its code is jumped to
  *addr = a;
  return "";
}

void jit_patch(std::vector<TInstr> &tc, const std::vector<JitRun> &runs, const std::vector<uint64_t> &addr) {
  for (size_t k = 0; k < runs.size(); k++) {
    uint32_t *w = tc[runs[k].pc].w;
    w[0] = TC_SLOT_JIT * TC_SLOT_BYTES;
    w[1] = uint32_t(addr[k]);
    w[2] = uint32_t(addr[k] >> 32);
    w[3] = w[4] = w[6] = w[7] = 0;
    w[5] = (runs[k].len - 1) * 32u;
  }
}

}  // namespace wb

// TEST hook (tests/test_jit.py, CPU): lower a module, pick its runs and assemble them for
// gfx950 without a device. Returns the number of runs, or -1 with the error in err.
extern "C" __attribute__((visibility("default"))) int wb_jit_check(const uint8_t *wasm, uint32_t len,
                                                                   uint32_t glog, uint32_t *instrs,
                                                                   char *err, uint32_t errlen) {
  wb::Program P;
  uint8_t ec = 0;
  std::string e = wb::load_program(wasm, len, P, &ec, false, nullptr, true, true);
  std::vector<wb::JitRun> runs;
  if (e.empty() && P.total_cells() > TC_VF_CELLS) e = "frame too large for V frames";
  // extra memories laid out at their minimum sizes (batch_api.cpp reserves more for grown ones)
  std::vector<uint32_t> xinfo;
  uint64_t words = 0;
  for (const auto &xm : P.xmems) {
    xinfo.push_back(uint32_t(words));
    xinfo.push_back(xm.min);
    words += uint64_t(xm.min) << 14;
  }
  if (e.empty()) {
    std::vector<DInstr> code = P.code;
    code.push_back(DInstr{0, 0, 0, 0});
    const std::vector<TInstr> tc = wb::build_threaded(P, code, true);
    runs = wb::jit_runs(P, tc);
    // debug listing: every DBC instruction (op, fields) with the SIMT run it belongs to
    if (const char *lst = getenv("WB_JIT_LIST"))
      if (FILE *f = fopen(lst, "w")) {
        static const char *const names[] = {
#define WB_NAME(x) #x,
            DBC_OPS(WB_NAME)
#undef WB_NAME
        };
        const std::vector<wb::JitRun> sr = wb::jit_runs(P, tc, true);
        std::vector<int> at(P.code.size(), -1);
        for (size_t k = 0; k < sr.size(); k++)
          for (uint32_t i = 0; i < sr[k].len; i++) at[sr[k].pc + i] = int(k);
        for (size_t pc = 0; pc < P.code.size(); pc++) {
          const DInstr &I = P.code[pc];
          const uint16_t op = uint16_t(I.w0 & 0x7FFFu);
          fprintf(f, "%4zu %s%-4s %-22s a=%u b=%u c=%u d=%d imm=0x%x cnt=%u\n", pc,
                  at[pc] >= 0 && sr[at[pc]].pc == pc ? "R" : " ",
                  at[pc] >= 0 ? std::to_string(at[pc]).c_str() : "-",
                  op < OP_DBC_NUM_OPS ? names[op] : "?", I.w1 & 0xFFFFu, I.w1 >> 16, I.w2 & 0xFFFFu,
                  int(int16_t(I.w2 >> 16)), I.w3, (I.w0 >> 16) & 0xFFu);
        }
        fclose(f);
      }
    if (instrs) {
      *instrs = 0;
      for (const auto &r : runs) *instrs += r.len;
    }
    // every flavour: plain runs, SIMT scheduling (KParams::simt, its own run choice) and
    // trip mode (its own run choice too)
    for (int simt = 0; simt < 3 && e.empty(); simt++) {
      if (simt) runs = wb::jit_runs(P, tc, true, simt == 2);
      if (runs.empty()) continue;
      std::vector<char> obj;
      // (a memory below kMadPages unless WB_JIT_CHECK_PAGES says otherwise: the 32-bit
      // granule addresses of trip stages assembled too)
      const char *cp = getenv("WB_JIT_CHECK_PAGES");
      const std::string src = wb::jit_source(P, runs, glog, nullptr, simt != 0, simt == 2, &xinfo,
                                             P.divergent_xmem ? 5u : 0u, cp ? uint32_t(atoi(cp)) : wb::kMadPages);
      if (const char *dump = getenv(simt == 2 ? "WB_JIT_DUMP_TRIP" : simt ? "WB_JIT_DUMP_SIMT" : "WB_JIT_DUMP"))
        if (FILE *f = fopen(dump, "w")) { fputs(src.c_str(), f); fclose(f); }
      e = src.empty() ? "no source" : wb::jit_compile(src, &obj);
    }
  }
  if (!e.empty()) {
    if (err && errlen) snprintf(err, errlen, "%s", e.c_str());
    return -1;
  }
  return int(runs.size());
}

// TEST hook (tests/test_jit.py, CPU): whether a SIMT context of this module runs trip mode
// (Program::divergent_mem or wb::trips_pay; WB_TRIP unset). 1 / 0, or -1 when it fails to load.
extern "C" __attribute__((visibility("default"))) int wb_trip_choice(const uint8_t *wasm, uint32_t len) {
  wb::Program P;
  uint8_t ec = 0;
  if (!wb::load_program(wasm, len, P, &ec).empty()) return -1;
  return P.divergent_mem || P.divergent_xmem || wb::trips_pay(P) ? 1 : 0;
}

// TEST hook (tests/test_depth_pick.py, CPU): whether the module counts as recursive for the
// depth-keyed SIMT pick (wb::recursive). 1 / 0, or -1 when it fails to load.
extern "C" __attribute__((visibility("default"))) int wb_recursive(const uint8_t *wasm, uint32_t len) {
  wb::Program P;
  uint8_t ec = 0;
  if (!wb::load_program(wasm, len, P, &ec).empty()) return -1;
  return wb::recursive(P) ? 1 : 0;
}
