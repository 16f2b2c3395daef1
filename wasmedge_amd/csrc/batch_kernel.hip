// batch_kernel.hip -- CDNA4 (gfx950) batched WebAssembly interpreter.
//
// One lane = one wasm instance; one wave = 64 instances executing the same module.
// Replaces the reference's Executor::execute dispatch loop (lib/executor/engine/
// engine.cpp:68-1638), StackManager (include/runtime/stackmgr.h) and MemoryInstance
// (include/runtime/instance/memory.h) for the batched path.
//
// Execution model
//  * wave-coherent dispatch: the wave fetches ONE 16-byte DBC instruction per step with
//    a scalar load (uniform pc), and executes it for the lanes whose pc matches.  When
//    all running lanes share a pc (the common, converged case) that costs one readlane +
//    one ballot; after divergence the wave runs the largest group of lanes sharing a pc,
//    which stops where it meets waiting lanes so they merge (KParams::sched = 0: the
//    minimum pc, which reconverges structured control flow at join points).
//  * frames: the CURRENT frame of every lane (globals + params + locals + operand cells)
//    lives in LDS, cell-major / lane-minor, so a cell access is one conflict-free
//    ds_read_b32/ds_write_b32 for the whole wave.  call spills the caller's live cells
//    to a lane-interleaved HBM call stack; return restores them (POST_CALL).
//  * linear memory: HBM, 4-byte words interleaved across the 64 lanes of a wave:
//    word w of lane l is at mem[(wave*W + w)*64 + l], so lanes touching the same address
//    coalesce into one 256-byte transaction.  Bounds and traps are per lane.
//  * counting: every dispatch adds its `cnt` (wasm instructions retired) to a per-lane
//    64-bit counter -- the reference's Statistics instruction count, exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <vector>

#include "dbc.h"
#include "kparams.h"


#include "dbc_ops.h"
#include "tc.h"
#include "tc_slots.h"

// The threaded dispatch core (gen_tc.py): hand-written gfx950 handlers. hipcc drops
// file-scope asm in device code, so the blob is the body of a kernel that is never
// launched (it would end at its first instruction); wb_exec_kernel enters and leaves
// the handlers through tc_run() below.
extern "C" __global__ void wb_tc_holder_kernel() {
  asm volatile("s_endpgm\n"
#include "tc_blob.inc"
               ::: "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69",
               "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80",
               "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91",
               "s92", "s93", "s94", "s95", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111",
               "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120",
               "v121", "v122", "v123", "v124", "v125", "v126", "v127", "vcc", "memory");
}
// The V-frame variant (frame cells in v128..v255, gen_tc.py VB) for wb_exec_vf_kernel.
extern "C" __global__ void __launch_bounds__(256) wb_vf_holder_kernel() {
  asm volatile("s_endpgm\n"
#include "tc_vblob.inc"
               ::: "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69",
               "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80",
               "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91",
               "s92", "s93", "s94", "s95", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111",
               "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120",
               "v121", "v122", "v123", "v124", "v125", "v126", "v127", "vcc", "memory");
}

// Minimum over the wave (all 64 lanes active), in VALU DPP steps instead of LDS permutes:
// row_shr 1/2/4/8 leave each row's prefix minimum in its lane 15, row_bcast:15 and
// row_bcast:31 fold rows 0-2 into rows 1-3, so lane 63 holds the wave minimum. Lanes whose
// DPP source is out of range keep the identity (`old` = ~0).
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  const int I = -1;
#define WB_DPP_MIN(ctrl, rmask)                                                            \
  do {                                                                                    \
    const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(I, (int)v, ctrl, rmask, 0xF, false); \
    v = t < v ? t : v;                                                                    \
  } while (0)
  WB_DPP_MIN(0x111, 0xF);   // row_shr:1
  WB_DPP_MIN(0x112, 0xF);   // row_shr:2
  WB_DPP_MIN(0x114, 0xF);   // row_shr:4
  WB_DPP_MIN(0x118, 0xF);   // row_shr:8
  WB_DPP_MIN(0x142, 0xA);   // row_bcast:15 into rows 1 and 3
  WB_DPP_MIN(0x143, 0xC);   // row_bcast:31 into rows 2 and 3
#undef WB_DPP_MIN
  return __builtin_amdgcn_readlane(v, 63);
}


// ======================================================================= interpreter
// Frame storage: cell-major / lane-minor LDS, so every cell access (a wave-uniform cell
// index decoded from the scalar-loaded instruction) is one conflict-free ds_read_b32.
// (Register-resident frames via s_set_gpr_idx were measured 10-45% slower on every
// workload -- see DESIGN.md "Frames" -- and removed.)
// Optional per-wave execution statistics (profiling builds: -DWB_STATS, see
// tools/sched_stats.py): scheduler rounds, fast runs and their active lanes, threaded-core
// entries, compiled-step dispatches, slow steps, and shader cycles per phase.
#ifdef WB_STATS
enum { ST_ROUNDS, ST_FAST, ST_LANES, ST_TC, ST_CPP, ST_SLOW, ST_CYC_SCHED, ST_CYC_FAST,
       ST_CYC_SLOW, ST_X_CALL, ST_X_RET, ST_X_POST, ST_X_BR, ST_X_OTHER, ST_CYC_TC, ST_TC_SCHED,
       ST_T0, ST_T1, ST_HW,   // the batch wave's start / end (s_memrealtime, 100 MHz) and where
                              // it ran (HW_ID: SIMD, CU, SE, XCC bits) -- tools/wave_timeline.py
       ST_N };
static_assert(ST_N <= 32, "per-wave stats stride is 32 (batch_api.cpp)");
// one relaxed atomic add per event from the first active lane (also inside divergent
// regions, where a per-wave count must be taken once); cycles in units of 16 clocks
#define WB_STAT_ADD(k, v)                                                              \
  do {                                                                                 \
    const uint64_t _m = __ballot(1);                                                   \
    if (stw && __lane_id() == (uint32_t)__builtin_ctzll(_m))                           \
      __hip_atomic_fetch_add(&stw[k], (uint64_t)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
  } while (0)
#define WB_NOW() (__builtin_amdgcn_s_memtime() >> 4)
#else
#define WB_STAT_ADD(k, v) ((void)0)
#define WB_NOW() 0ull
#endif

typedef __attribute__((address_space(3))) uint32_t lds_u32;
struct LdsFrame {
  lds_u32 *fr;   // LDS-typed so the compiler knows frame cells never alias HBM
  __device__ __forceinline__ uint32_t get(uint32_t i) const { return fr[i << 6]; }
  __device__ __forceinline__ void set(uint32_t i, uint32_t v) { fr[i << 6] = v; }
  __device__ __forceinline__ uint32_t lds_addr() const { return (uint32_t)(uintptr_t)fr; }
};

// Frames too large for LDS (KParams::hframe): cell-major, lane-minor in HBM like linear
// memory's word interleave, [wave][cell][64]; the compiled step only (no threaded core).
struct HbmFrame {
  uint32_t *fr;
  __device__ __forceinline__ uint32_t get(uint32_t i) const { return fr[(size_t)i << 6]; }
  __device__ __forceinline__ void set(uint32_t i, uint32_t v) { fr[(size_t)i << 6] = v; }
  __device__ __forceinline__ uint32_t lds_addr() const { return 0u; }
};

// Run the threaded core from uniform pc `pc` for the lanes in EXEC until it meets an
// instruction it cannot finish for all of them (reason 0: the C++ step executes that
// instruction next), or reaches `other` / the count limit (reason 1: back to the
// scheduler). Returns the new uniform pc; *ncnt = wasm instructions retired.
// Register contract: gen_tc.py (s60-s93, v104-v127 belong to the core).
// (gsp is read-write: only the run's lanes (EXEC) take the core's value, the waiting
// lanes keep theirs)
#define TC_RUN_ASM(ENTRY, ...) \
  asm volatile( \
      "s_mov_b32 s60, %[clo]\n\t" \
      "s_mov_b32 s61, %[chi]\n\t" \
      "s_lshl_b32 s62, %[pc], 5\n\t" \
      "s_mov_b32 s63, %[oth]\n\t" \
      "s_mov_b32 s64, %[lim]\n\t" \
      "s_mov_b32 s65, 0\n\t" \
      "v_mov_b32 v104, %[fr]\n\t" \
      "v_mov_b32 v105, %[pages]\n\t" \
      "v_mov_b32 v106, %[mlo]\n\t" \
      "v_mov_b32 v107, %[mhi]\n\t" \
      "v_mov_b32 v102, %[gsp]\n\t" \
      "v_mov_b32 v101, %[hwm]\n\t" \
      "v_mov_b32 v103, %[stk]\n\t" \
      "v_mov_b32 v99, %[msh]\n\t" \
      "v_add_u32_e32 v100, 6, v99\n\t" \
      "s_mov_b32 s93, %[slds]\n\t" \
      "v_mov_b32 v94, %[llo]\n\t" \
      "v_mov_b32 v95, %[lhi]\n\t" \
      "v_mov_b32 v96, %[glo]\n\t" \
      "v_mov_b32 v97, %[ghi]\n\t" \
      "s_mov_b32 s94, %[vsync]\n\t" \
      "s_mov_b32 s95, %[low]\n\t" \
      "s_getpc_b64 s[66:67]\n" \
      "Ltc_ret_%=:\n\t" \
      "s_add_u32 s66, s66, Ltc_back_%= - Ltc_ret_%=\n\t" \
      "s_addc_u32 s67, s67, 0\n\t" \
      "s_getpc_b64 s[68:69]\n\t" \
      "s_add_u32 s68, s68, " ENTRY "@rel32@lo+4\n\t" \
      "s_addc_u32 s69, s69, " ENTRY "@rel32@hi+12\n\t" \
      "s_setpc_b64 s[68:69]\n" \
      "Ltc_back_%=:\n\t" \
      "s_lshr_b32 %[npc], s62, 5\n\t" \
      "s_mov_b32 %[cnt], s65\n\t" \
      "s_mov_b32 %[why], s92\n\t" \
      "v_mov_b32 %[gsp], v102\n\t" \
      "v_mov_b32 %[glo], v96\n\t" \
      "v_mov_b32 %[ghi], v97\n\t" \
      "v_mov_b32 %[hwm], v101" \
      : [npc] "=s"(npc), [cnt] "=s"(cnt), [why] "=s"(why), [gsp] "+v"(gsp), [hwm] "+v"(hwm), \
        [glo] "+v"(glo), [ghi] "+v"(ghi) \
      : [clo] "s"(clo), [chi] "s"(chi), [pc] "s"(pc), [oth] "s"(oth), [lim] "s"(lim), [fr] "v"(fr), \
        [pages] "v"(pages), [mlo] "v"(mlo), [mhi] "v"(mhi), [stk] "v"(stk), [msh] "s"(msh), \
        [slds] "s"(slds), [vsync] "s"(vsync), [low] "s"(lw), [llo] "s"(llo), [lhi] "s"(lhi) \
      : "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", \
        "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", \
        "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95", \
        "v94", "v95", "v96", "v97", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", \
        "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", \
        "v124", "v125", "v126", "v127", "vcc", "scc", "memory", ##__VA_ARGS__);

// VF: the V-frame core (wb_vf_entry): it loads the frames of the lanes in ALL (s[96:97])
// into v128.. on entry, runs the group in s[74:75], and stores the frames back on exit
// (vsync = (TC_VF_CELLS - frame cells) * 8, gen_tc.py VSYNC). It returns the group that
// left in s[74:75] and, for every lane in ALL, its pc (v92) and the wasm instructions it
// retired (v93): in SIMT mode (KParams::simt) the compiled runs schedule the lanes among
// themselves (jit.cpp Lsched), otherwise ALL = the group = EXEC throughout. The caller's
// EXEC (`ex`) is restored at the end. s[98:99] = the wave's block of the memories past the
// first (KParams::xmem; the compiled XLD / XST, jit.cpp emit_xmem), 0 without them.
#define TC_RUN_VF_ASM(...) \
  asm volatile( \
      "s_mov_b32 s60, %[clo]\n\t" \
      "s_mov_b32 s61, %[chi]\n\t" \
      "s_lshl_b32 s62, %[pc], 5\n\t" \
      "s_mov_b32 s63, %[oth]\n\t" \
      "s_mov_b32 s64, %[lim]\n\t" \
      "s_mov_b32 s65, 0\n\t" \
      "s_mov_b64 s[96:97], %[all]\n\t" \
      "s_mov_b64 s[74:75], %[grp]\n\t" \
      "v_mov_b32 v104, %[fr]\n\t" \
      "v_mov_b32 v105, %[pages]\n\t" \
      "v_mov_b32 v106, %[mlo]\n\t" \
      "v_mov_b32 v107, %[mhi]\n\t" \
      "v_mov_b32 v102, %[gsp]\n\t" \
      "v_mov_b32 v101, %[hwm]\n\t" \
      "v_mov_b32 v103, %[stk]\n\t" \
      "v_mov_b32 v99, %[msh]\n\t" \
      "v_add_u32_e32 v100, 6, v99\n\t" \
      "v_mov_b32 v92, %[vpc]\n\t" \
      "v_mov_b32 v93, 0\n\t" \
      "s_mov_b32 s93, %[slds]\n\t" \
      "v_mov_b32 v94, %[llo]\n\t" \
      "v_mov_b32 v95, %[lhi]\n\t" \
      "v_mov_b32 v96, %[glo]\n\t" \
      "v_mov_b32 v97, %[ghi]\n\t" \
      "s_mov_b32 s94, %[vsync]\n\t" \
      "s_mov_b32 s95, %[low]\n\t" \
      "s_mov_b32 s98, %[xlo]\n\t" \
      "s_mov_b32 s99, %[xhi]\n\t" \
      "s_mov_b64 exec, s[96:97]\n\t" \
      "s_getpc_b64 s[66:67]\n" \
      "Ltc_ret_%=:\n\t" \
      "s_add_u32 s66, s66, Ltc_back_%= - Ltc_ret_%=\n\t" \
      "s_addc_u32 s67, s67, 0\n\t" \
      "s_getpc_b64 s[68:69]\n\t" \
      "s_add_u32 s68, s68, wb_vf_entry@rel32@lo+4\n\t" \
      "s_addc_u32 s69, s69, wb_vf_entry@rel32@hi+12\n\t" \
      "s_setpc_b64 s[68:69]\n" \
      "Ltc_back_%=:\n\t" \
      "s_lshr_b32 %[npc], s62, 5\n\t" \
      "s_mov_b32 %[cnt], s65\n\t" \
      "s_mov_b32 %[why], s92\n\t" \
      "s_mov_b32 %[noth], s63\n\t" \
      "s_mov_b32 %[nlow], s95\n\t" \
      "s_mov_b64 %[ngrp], s[74:75]\n\t" \
      "v_mov_b32 %[gsp], v102\n\t" \
      "v_mov_b32 %[glo], v96\n\t" \
      "v_mov_b32 %[ghi], v97\n\t" \
      "v_mov_b32 %[vpc], v92\n\t" \
      "v_mov_b32 %[vcnt], v93\n\t" \
      "v_mov_b32 %[hwm], v101\n\t" \
      "s_mov_b64 exec, %[ex]" \
      /* (early-clobber outputs: they are written before `ex` is read) */ \
      : [npc] "=&s"(npc), [cnt] "=&s"(cnt), [why] "=&s"(why), [noth] "=&s"(noth), [nlow] "=&s"(nlow), \
        [ngrp] "=&s"(ngrp), [gsp] "+v"(gsp), [hwm] "+v"(hwm), [glo] "+v"(glo), [ghi] "+v"(ghi), \
        [vpc] "+v"(vpc), [vcnt] "=&v"(vcnt) \
      : [clo] "s"(clo), [chi] "s"(chi), [pc] "s"(pc), [oth] "s"(oth), [lim] "s"(lim), [fr] "v"(fr), \
        [pages] "v"(pages), [mlo] "v"(mlo), [mhi] "v"(mhi), [stk] "v"(stk), [msh] "s"(msh), \
        [slds] "s"(slds), [vsync] "s"(vsync), [low] "s"(lw), [llo] "s"(llo), [lhi] "s"(lhi), \
        [all] "s"(all), [grp] "s"(grp), [ex] "s"(ex), [xlo] "s"(xlo), [xhi] "s"(xhi) \
      : "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", \
        "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", \
        "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95", "s96", "s97", \
        "s98", "s99", \
        "v92", "v93", "v94", "v98", "v95", "v96", "v97", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", \
        "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", \
        "v124", "v125", "v126", "v127", "vcc", "scc", "memory", ##__VA_ARGS__);
#define TC_VREGS "v128", "v129", "v130", "v131", "v132", "v133", "v134", "v135", "v136", "v137", \
  "v138", "v139", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147", "v148", "v149", \
  "v150", "v151", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159", "v160", "v161", \
  "v162", "v163", "v164", "v165", "v166", "v167", "v168", "v169", "v170", "v171", "v172", "v173", \
  "v174", "v175", "v176", "v177", "v178", "v179", "v180", "v181", "v182", "v183", "v184", "v185", \
  "v186", "v187", "v188", "v189", "v190", "v191", "v192", "v193", "v194", "v195", "v196", "v197", \
  "v198", "v199", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", \
  "v210", "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", \
  "v222", "v223", "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", \
  "v234", "v235", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", \
  "v246", "v247", "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255"
// What a SIMT-mode core call (VF) hands back besides the group's pc: the group, its
// stop pcs, and for every lane in ALL its pc and retired instructions.
struct SimtOut {
  uint64_t grp;
  uint32_t oth, low, vpc, vcnt;
};
template <bool VF>
__device__ __forceinline__ uint32_t tc_run(const void *tcode, uint32_t pc, uint32_t other, uint32_t low,
                                           uint32_t fr, uint32_t pages, const uint32_t *mem, uint32_t g,
                                           uint32_t &gsp, uint32_t &hwm, uint32_t stk, uint32_t slds,
                                           uint32_t vsync, uint64_t &gas, uint64_t gas_limit,
                                           uint32_t *ncnt, uint32_t *reason, uint32_t lim,
                                           SimtOut *so = nullptr, uint64_t all = 0, uint64_t grp = 0,
                                           uint32_t vpc = 0, uint64_t xbase = 0) {
  uint32_t npc, cnt, why;
  // metered contexts: the lane's gas total in v[96:97] and the limit in v[94:95] for the
  // compiled runs (jit.cpp), which price themselves; handlers never touch them
  uint32_t glo = (uint32_t)gas, ghi = (uint32_t)(gas >> 32);
  const uint32_t llo = __builtin_amdgcn_readfirstlane((uint32_t)gas_limit);
  const uint32_t lhi = __builtin_amdgcn_readfirstlane((uint32_t)(gas_limit >> 32));
  const uint32_t oth = __builtin_amdgcn_readfirstlane(other >= (1u << 26) ? 0xFFFFFFFFu : other << 5);
  const uint32_t lw = __builtin_amdgcn_readfirstlane(low >= (1u << 26) ? 0xFFFFFFFFu : low << 5);
  const uint64_t m = (uint64_t)(uintptr_t)mem;
  const uint32_t msh = 2u + g;   // gen_tc.py MSH1 (MSH2 = MSH1 + 6)
  const uint32_t mlo = (uint32_t)m, mhi = (uint32_t)(m >> 32);
  const uint64_t cp = (uint64_t)(uintptr_t)tcode;   // as two words: no aligned pair needed
  const uint32_t clo = (uint32_t)cp, chi = (uint32_t)(cp >> 32);
  // all of these are wave-uniform; readfirstlane keeps them in SGPRs even where the
  // compiler's divergence analysis cannot prove it (profiling builds)
  pc = __builtin_amdgcn_readfirstlane(pc);
  if constexpr (VF) {
    // (the caller's EXEC; without SIMT the core runs exactly it: ALL = the group = EXEC)
    const uint64_t ex = __builtin_amdgcn_read_exec();
    if (!so) all = grp = ex;
    const uint32_t xlo = __builtin_amdgcn_readfirstlane((uint32_t)xbase);
    const uint32_t xhi = __builtin_amdgcn_readfirstlane((uint32_t)(xbase >> 32));
    uint32_t noth, nlow, vcnt;
    uint64_t ngrp;
    TC_RUN_VF_ASM(TC_VREGS);
    if (so) *so = SimtOut{ngrp, noth, nlow, vpc, vcnt};
  } else {
    TC_RUN_ASM("wb_tc_entry");
  }
  gas = (uint64_t)glo | ((uint64_t)ghi << 32);
  *ncnt = cnt;
  *reason = why;
  return npc;
}

// PG: the module can grow past the reserved layout (KParams::grow_host), so a lane's memory
// may have pool pages: only then do the per-lane step's accesses go through the page table
// and memory.size / memory.grow read the size from LS_PAGES (the fast paths never change).
template <bool VF, bool PG, class Frame>
__device__ __forceinline__ void interp(const KParams &p, Frame &F, const uint32_t inst,
                                       uint32_t *const gs, const GMem mem,
                                       uint32_t *const ls, uint32_t *const fs,
                                       lds_u32 *const stk) {
  // the bytecode is read through the constant address space so every fetch is one
  // scalar s_load_dwordx4 (uniform pc) instead of a vector load + readfirstlanes
  typedef uint32_t w4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(4))) const w4 *cptr;
  const cptr code = (cptr)p.code;

#define R32(x) F.get((uint32_t)(x))
#define R64(x) ((uint64_t)F.get((uint32_t)(x)) | ((uint64_t)F.get((uint32_t)(x) + 1) << 32))
#define W32(c, v) F.set((uint32_t)(c), (uint32_t)(v))
#define W64(c, v) do { const uint64_t _v = (v); F.set((uint32_t)(c), (uint32_t)_v); F.set((uint32_t)(c) + 1, (uint32_t)(_v >> 32)); } while (0)
#define W128(c, v) do { for (int _k = 0; _k < 4; _k++) F.set((uint32_t)(c) + _k, (v)[_k]); } while (0)
#define WLOOP(c, v) F.set((uint32_t)(c), (uint32_t)(v))
// Call stack: slots [0, gs_lds) in LDS (`stk`, cell-major like frames), the rest in HBM
// (`gs`, lane-interleaved). The fast loop only touches the LDS part (GS_FAST checks it
// per wave); the per-lane step handles either.
  const uint32_t S_lds = p.gs_lds;
#define GS_RD(s) ((uint32_t)(s) < S_lds ? stk[(uint32_t)(s) << 6] : gs[(size_t)((uint32_t)(s) - S_lds) << 6])
#define GS_WR(s, v) do { const uint32_t _s = (s), _v = (v); \
    if (_s < S_lds) stk[_s << 6] = _v; else gs[(size_t)(_s - S_lds) << 6] = _v; } while (0)
#define GS_FAST(hi) ((hi) <= S_lds)
#define GSF_BASE(s) (&stk[(uint32_t)(s) << 6])
#define GS_PTR lds_u32 *const
#define GS_CPTR const lds_u32 *const

#define LS(slot) ls[(size_t)(slot) << 6]
  // per-lane tables: entries lane-interleaved like memory, sizes + dropped elems in LS
  uint32_t *const lt = p.ltab ? p.ltab + (size_t)(inst >> 6) * p.tab_words * 64u + (inst & 63u) : nullptr;
#define TSIZE(t) LS(p.ls_tab + (t))
#define TENT(t, i) lt[(size_t)(p.tabinfo[2u * (t)] + (i)) << 6]
#define WB_TWIDEN(t, want) ((void)0)   // (a grow past the capacity parks before the step)
// dropped element segments: mask words after the table sizes; dropped data segments: the
// first 32 in `dropped` (LS_DROPPED), the rest in mask words at ls_drop_ext (slow paths only)
#define ELEM_DROPPED(e) ((LS(p.ls_tab + p.ntables + ((e) >> 5)) >> ((e) & 31u)) & 1u)
#define SET_ELEM_DROPPED(e) (LS(p.ls_tab + p.ntables + ((e) >> 5)) |= 1u << ((e) & 31u))
#define DATA_DROPPED(s) ((s) < 32u ? (dropped >> (s)) & 1u : (LS(p.ls_drop_ext + ((s) >> 5) - 1u) >> ((s) & 31u)) & 1u)
#define SET_DATA_DROPPED(s) do { const uint32_t _s = (s); \
    if (_s < 32u) dropped |= 1u << _s; else LS(p.ls_drop_ext + (_s >> 5) - 1u) |= 1u << (_s & 31u); } while (0)
  uint32_t status = inst < p.n ? WB_STATUS_RUNNING : WB_STATUS_OK;
  // `pages` = the lane's pages in the reserved layout, min(its memory size, rpages): the
  // bound of every fast path. The size itself is LS_PAGES (memory.grow writes it there),
  // read where it can exceed rpages (MEM_PAGES).
  uint32_t pc = p.entry_pc, gsp = 0, pages = min(LS(LS_PAGES), p.rpages), dropped = LS(LS_DROPPED);
  // (addressed from the kernel arguments, not `ls`: no extra pointer live through the loop)
#define LS_PAGES_REF p.lstate[((size_t)__builtin_amdgcn_readfirstlane(inst >> 6) * p.ls_slots + LS_PAGES) * 64u + lane]
#define MEM_PAGES (PG && pages >= p.rpages ? LS_PAGES_REF : pages)
  // one past the highest memory byte written since instantiation: Reset re-initialises
  // only [0, hwm) of each lane (plus the image), the rest is still the zero it was given
  uint32_t hwm = LS(LS_HWM);
#define WB_MARK(ea, n) (hwm = max(hwm, (uint32_t)min((uint64_t)(ea) + (uint64_t)(n), 0xFFFFFFFFull)))
  // memories past the first (MultiMemories, KParams::xmem): granules of 4 << xlog bytes
  // interleaved over the wave's lanes; the per-lane step (dbc_step.inc XLD ... XMEM_COPY)
  // and the compiled XLD / XST (jit.cpp emit_xmem) reach them
#define XMEM(k) GMem{p.xmem + ((size_t)(inst >> 6) * p.xwords + p.xinfo[2u * ((k) - 1u)]) * 64u + \
                     ((inst & 63u) << p.xlog), p.xlog}
#define XPAGES(k) p.xpages[(size_t)((k) - 1u) * p.xstride + inst]
#define XLIMIT(k) p.xinfo[2u * ((k) - 1u) + 1u]
#define XGROW(k, cur, n) (XPAGES(k) = (cur) + (n))
  uint64_t count = 0;
  // the running gas total (metered runs): kept in the instance state between launches
  uint64_t cost = (uint64_t)LS(LS_COST) | ((uint64_t)LS(LS_COST + 1) << 32);
  const uint32_t istatus = LS(LS_ISTATUS);
  if (status == WB_STATUS_RUNNING && istatus) status = istatus;   // instance never came up
  for (uint32_t c = 0; c < p.global_cells; c++) F.set(c, LS(LS_GLOBALS + c));
  uint32_t ycall = 0, ybase = 0;   // host import being called when the lane yields
  bool active = inst < p.n;   // the lane has an instance (partial waves)
  if (p.resume) {
    // continue a lane parked at a host import: frame from fsave, the host function's
    // results (hcall = their cell count, ~0 = the host ended the lane) into its cells
    const uint32_t rpc = LS(LS_RPC);
    const bool parked = status == WB_STATUS_RUNNING && rpc != 0xFFFFFFFFu;
    const uint32_t nres = parked ? p.hcall[inst] : 0xFFFFFFFFu;
    active = parked && nres != 0xFFFFFFFFu;
    if (parked) LS(LS_RPC) = 0xFFFFFFFFu;
    if (active) {
      pc = rpc;
      gsp = LS(LS_GSP);
      count = p.counts[inst];
      for (uint32_t c = p.global_cells; c < p.total_cells; c++) F.set(c, fs[(size_t)c << 6]);
      for (uint32_t k = 0; k < gsp && k < S_lds; k++) stk[k << 6] = fs[(size_t)(p.total_cells + k) << 6];
      const uint32_t base = LS(LS_HBASE);
      for (uint32_t k = 0; k < nres; k++) F.set(base + k, p.hbuf[(size_t)inst * p.hb_cells + k]);
    } else {
      status = WB_STATUS_OK;
    }
  } else if (status == WB_STATUS_RUNNING) {
    if (fs) LS(LS_RPC) = 0xFFFFFFFFu;   // a fresh invocation: nothing parked
    const uint32_t *prm = p.params + (size_t)inst * p.param_cells;
    for (uint32_t c = 0; c < p.param_cells; c++) F.set(p.global_cells + c, prm[c]);
    GS_WR(0u, DBC_EXIT_PC);   // return record of the entry frame: pc = EXIT
    gsp = 1;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#ifdef WB_STATS
  if (p.stats && !p.resume && __lane_id() == (uint32_t)__builtin_ctzll(__ballot(1))) {
    uint64_t *const sw = p.stats + (size_t)(inst >> 6) * 32u;
    sw[ST_T0] = t0;
    sw[ST_HW] = __builtin_amdgcn_s_getreg((4 << 0) | (31 << 11)) |   // HW_REG_HW_ID (gfx9 id 4)
                ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (31 << 11)) << 32);   // XCC_ID
  }
#endif
  uint64_t tpoll = t0 - 1000u;   // the last read of the interrupt flag (100 MHz ticks)
#ifdef WB_STATS
  uint64_t *const stw = p.stats ? p.stats + (size_t)(inst >> 6) * 32u : nullptr;
#endif
  const uint32_t lane = __lane_id();
  const uint32_t fr_lds = F.lds_addr();   // this lane's cell 0, LDS byte address
  const uint32_t stk_lds = (uint32_t)(uintptr_t)stk;   // its call-stack slot 0
  // the wave's block of the memories past the first (XMEM below; the compiled XLD / XST)
  const uint64_t xbase = p.n_xmem ? (uint64_t)(uintptr_t)(p.xmem + (size_t)(inst >> 6) * p.xwords * 64u) : 0;

  for (;;) {
    // ---- schedule: which group of lanes (same pc) runs next; `other` = the lowest pc
    // of the waiting lanes above it, `low` = the lowest pc of all waiting lanes.
    const uint64_t runmask = __ballot(status == WB_STATUS_RUNNING);
    if (!runmask) break;
    [[maybe_unused]] const uint64_t ts0 = WB_NOW();
    WB_STAT_ADD(ST_ROUNDS, 1);
    uint32_t pcs = __builtin_amdgcn_readlane(pc, (uint32_t)__builtin_ctzll(runmask));
    uint64_t act = __ballot(status == WB_STATUS_RUNNING && pc == pcs);
    uint32_t other = 0xFFFFFFFFu, low = 0xFFFFFFFFu;
    if (act != runmask) {
      // the lowest pc first: structured control flow puts join points above both arms,
      // so min-pc scheduling reconverges divergent lanes. But a short scan loop at a low
      // pc (`while (a[i] < p) i++`: data-dependent trip counts) then holds every lane
      // waiting past its exit until its slowest lane leaves: the scan loops of a Hoare
      // partition ran 3.5 lanes per dispatch. So when the min-pc lanes are in a scan
      // loop (the lowering's loop table: innermost loops < 8 instructions), the largest
      // group waiting past that loop runs instead if it has >= sched x their lanes;
      // those lanes come back round (outer loop, recursion) and merge
      // (tools/sched_study.py: C3 3.5 -> 14.3 lanes per dispatch, C4/C5 unchanged;
      // measured C3 3.9e10 -> 9.1e10 instr/s). A group stops at the next waiting pc
      // above it (`other`), and after a jump to or below the lowest waiting pc (`low`)
      // at that one.
      pcs = wave_min_u32(status == WB_STATUS_RUNNING ? pc : 0xFFFFFFFFu);
      act = __ballot(status == WB_STATUS_RUNNING && pc == pcs);
      bool moved = false;
      if (p.sched) {
        typedef __attribute__((address_space(4))) const uint32_t *cu32;
        const uint32_t lh = ((cu32)p.loops)[2 * pcs], le = ((cu32)p.loops)[2 * pcs + 1];
        const uint32_t nmin = (uint32_t)__builtin_popcountll(act);
        uint32_t need = nmin * p.sched > nmin ? nmin * p.sched : nmin + 1;
        uint64_t rem = lh == 0xFFFFFFFFu ? 0 : __ballot(status == WB_STATUS_RUNNING && pc > le);
        while (rem && (uint32_t)__builtin_popcountll(rem) >= need) {
          const uint32_t q = __builtin_amdgcn_readlane(pc, (uint32_t)__builtin_ctzll(rem));
          const uint64_t m = __ballot(status == WB_STATUS_RUNNING && pc == q);
          const uint32_t k = (uint32_t)__builtin_popcountll(m);
          if (k >= need) { need = k + 1; pcs = q; act = m; moved = true; }
          rem &= ~m;
        }
      }
      if (act != runmask) {
        low = wave_min_u32(status == WB_STATUS_RUNNING && pc != pcs ? pc : 0xFFFFFFFFu);
        other = moved ? wave_min_u32(status == WB_STATUS_RUNNING && pc > pcs ? pc : 0xFFFFFFFFu) : low;
      }
    }
    // The core's budget per call (instructions of the groups it runs; trip mode: 256 per
    // trip): it returns to this loop, which checks the limits and the interrupt flag, at
    // least every 2^20 instructions -- and, under MaxSteps, before any running lane could
    // pass its budget by more than the run it is in
    uint32_t core_lim = 1u << 20;
    if (p.max_steps < (1ull << 62)) {
      const uint64_t rem = count < p.max_steps ? p.max_steps - count : 1;
      const uint32_t r32 = (uint32_t)min(rem, (uint64_t)core_lim);
      core_lim = max(1u, wave_min_u32(status == WB_STATUS_RUNNING ? r32 : 0xFFFFFFFFu));
    }
    bool slow = false;   // the run stopped at an instruction that needs the slow step
    bool first = false;  // SIMT: the core left the group before a HOT instruction
    if constexpr (VF) {
      if (p.simt && (code[pcs].x & DBC_HOT)) {
        // SIMT mode: every running lane enters the core (EXEC is the whole wave here);
        // the compiled runs pick groups themselves and hand back each lane's pc and
        // retired instructions, and the group (if any) whose next instruction the C++
        // step must execute (reason 0)
        WB_STAT_ADD(ST_TC, 1);
        [[maybe_unused]] const uint64_t tt0 = WB_NOW();
        SimtOut so;
        uint32_t ncnt, why;
        const uint32_t gpc = tc_run<VF>(p.tcode, pcs, other, low, fr_lds, pages, mem.p, mem.g, gsp, hwm,
                                        stk_lds, S_lds, (TC_VF_CELLS - p.total_cells) * 8u, cost, ~0ull,
                                        &ncnt, &why, core_lim, &so, runmask, act, pc, xbase);
        WB_STAT_ADD(ST_CYC_TC, WB_NOW() - tt0);
        if (status == WB_STATUS_RUNNING) {
          pc = so.vpc;
          count += (uint64_t)(int64_t)(int32_t)so.vcnt;   // (a taken jump's count can be < 0)
        }
        if (why) {   // the core's budget is spent: nothing for the C++ step this round
          WB_STAT_ADD(ST_TC_SCHED, 1);
          act = 0;
        } else {
          act = so.grp;
          pcs = gpc;
          other = so.oth == 0xFFFFFFFFu ? 0xFFFFFFFFu : so.oth >> 5;
          low = so.low == 0xFFFFFFFFu ? 0xFFFFFFFFu : so.low >> 5;
          first = true;
        }
      }
    }
    [[maybe_unused]] const uint64_t ts1 = WB_NOW();
    WB_STAT_ADD(ST_CYC_SCHED, ts1 - ts0);
    WB_STAT_ADD(ST_FAST, 1);
    WB_STAT_ADD(ST_LANES, __builtin_popcountll(act));
    // (select by the ballot bit, not by `pc == pcs`: under that condition the compiler
    // would substitute the per-lane pc for pcs and make the whole run divergent)
    if ((act >> lane) & 1u) {
      // ================================================================ fast run
      // EXEC = act for the whole run. Every branch inside is wave-uniform (the compiler
      // leaves the dispatch tree as plain scalar branches); a dispatch continues with
      //   fall out of the switch      -> k_next: pcs + 1
      //   JUMP(t, tc)                 -> uniform jump (tc = taken-branch count correction)
      //   BRANCH(c, t, tc)            -> all lanes agree: stay; split: leave the run
      //   JUMP_LANE(t, tc)            -> per-lane target: stay when uniform, else leave
      //   TRAP(code) + TRAP_CHECK()   -> leave when any lane trapped
      //   SLOW_IF(c) / SLOW_OP()      -> leave before any side effect; the slow step
      //                                  below executes this instruction per lane
      // Per-lane state (pc, status, count corrections) changes only on exit paths.
#define WB_FAST 1
#define JUMP(t, tc) do { sc += cnt8 + (uint32_t)(tc); pcs = (t); goto k_jump; } while (0)
#define BRANCH(c, t, tc) do { const bool _c = (c); const uint64_t _m = __ballot(_c); \
    if (_m == act) JUMP(t, tc); \
    if (_m) { xpc = _c ? (uint32_t)(t) : pcs + 1; xadj = _c ? (int32_t)(tc) : 0; goto k_exit; } \
    goto k_next; } while (0)
#define JUMP_LANE(t, tc) do { const uint32_t _t = (t); const int32_t _tc = (tc); \
    const uint32_t _n0 = __builtin_amdgcn_readfirstlane(_t); \
    const int32_t _c0 = __builtin_amdgcn_readfirstlane(_tc); \
    if (__ballot(_t == _n0 && _tc == _c0) == act) JUMP(_n0, _c0); \
    xpc = _t; xadj = _tc; goto k_exit; } while (0)
#define WB_UNIFORM(x) __builtin_amdgcn_readfirstlane(x)   // (dbc_step.inc: a wave-uniform value)
#define TRAP(code) (tcode = (code))
#define FINISH() (tcode = WB_TCODE_DONE)
#define EXIT_IF_TRAPPED(t) do { if (__ballot(tcode != 0)) { xpc = (t); xadj = 0; goto k_exit; } } while (0)
#define TRAP_CHECK() EXIT_IF_TRAPPED(pcs + 1)
#define SLOW_OP() goto k_slow
#define SLOW_IF(c) do { if (__ballot(c)) goto k_slow; } while (0)
#define HOST_YIELD(f, base) SLOW_OP()
#define MEM_BYTES ((uint64_t)pages << 16)
#define WB_GROW(cur, n, res) ((void)0)
      uint32_t sc = 0, tick = 1024, xpc = 0, xpost = 0, tcode = 0;
      int32_t xadj = 0;
      uint64_t scost = 0;   // gas of the run so far (metered runs; wave-uniform)
      uint64_t asc = 0;     // instructions retired inside the threaded core
      w4 I = code[pcs];
      for (;;) {
        if (!(VF && p.simt) && p.tcode && (I.x & DBC_HOT)) {
          // hand the run to the threaded core; it returns at an instruction this
          // C++ step must execute (reason 0), or for the scheduler (reason 1)
          uint32_t ncnt, why;
          WB_STAT_ADD(ST_TC, 1);
          [[maybe_unused]] const uint64_t tt0 = WB_NOW();
          // (metered: the run's gas so far joins the lanes' totals first, jit.cpp prices
          // the compiled runs against the limit itself)
          cost += scost;
          scost = 0;
          pcs = tc_run<VF>(p.tcode, pcs, other, low, fr_lds, pages, mem.p, mem.g, gsp, hwm, stk_lds, S_lds,
                            (TC_VF_CELLS - p.total_cells) * 8u, cost,
                            p.cost_off ? p.cost_limit : ~0ull, &ncnt, &why, core_lim, nullptr, 0, 0, 0, xbase);
          // (sign-extended: a core call that only takes a jump whose count correction is
          // negative -- a `br` out of blocks, cnt 1 + tcnt -2 -- retires -1 instructions)
          asc += (uint64_t)(int64_t)(int32_t)ncnt;
          WB_STAT_ADD(ST_CYC_TC, WB_NOW() - tt0);
          if (why) WB_STAT_ADD(ST_TC_SCHED, 1);
          if (why) { xpc = pcs; tcode = 0; xadj = 0; break; }   // = k_leave
          I = code[pcs];
#ifdef WB_STATS
          {
            const uint32_t xo = I.x & 0x7FFFu;
            WB_STAT_ADD(xo == OP_CALL || xo == OP_CALL_INDIRECT ? ST_X_CALL : xo == OP_RET ? ST_X_RET
                        : xo == OP_POST_CALL ? ST_X_POST : (xo >= OP_JMP && xo <= OP_BR_TABLE) ? ST_X_BR
                        : ST_X_OTHER, 1);
            // which op made the core exit: a histogram after the per-wave counters
            if (stw && __lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)))
              __hip_atomic_fetch_add(&p.stats[(size_t)((p.n + 63) >> 6) * 32u + (xo & 1023u)], 1ull,
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
#endif
        }
        const uint32_t w0 = I.x, w1 = I.y, w2 = I.z, w3 = I.w;
        // Prefetch the fall-through successor only after I is resident: SMEM returns out
        // of order, so a use of I issued after the prefetch would wait for both.
        asm volatile("" ::"s"(w0), "s"(w1), "s"(w2), "s"(w3));
        const w4 In = code[pcs + 1];
        const uint32_t op = w0 & 0x7FFFu;
        const uint32_t cnt8 = (w0 >> 16) & 0xFFu, post8 = (w0 >> 24) & 0x7Fu;
        const int32_t tcnt = (int32_t)(int16_t)(w2 >> 16);
        WB_STAT_ADD(ST_CPP, 1);
        // metered (the threaded core is off, see launch_once): only straight-line
        // dispatches stay in the run, each priced at the full cost of the instructions it
        // retires; one that branches or may trap, or whose cost could reach the limit (or
        // wrap the sum), runs in the exact slow step
        uint64_t dfull = 0;
        if (p.cost_off) {
          typedef __attribute__((address_space(4))) const uint32_t *cu32;
          typedef __attribute__((address_space(4))) const uint64_t *cu64;
          dfull = cnt8 ? ((cu64)p.cost_pool)[((cu32)p.cost_off)[pcs] + cnt8 - 1] : 0;
          const uint64_t need = scost + dfull;
          SLOW_IF((w0 & DBC_CTL) || need < scost || cost > p.cost_limit || p.cost_limit - cost < need);
        }
        // SIMT: a HOT instruction goes back to the core (with every running lane), but
        // the one the core left the group before runs here
        if (VF && p.simt && (w0 & DBC_HOT) && !first) goto k_leave;
        first = false;
        switch (op) {
#define WB_XMEM_ON 0
#include "dbc_step.inc"
#undef WB_XMEM_ON
        }
      k_next:
        sc += cnt8;
        scost += dfull;
        pcs += 1;
        if (pcs >= other) { xpc = pcs; goto k_leave; }   // reached a waiting lane
        I = In;
        continue;
      k_jump:
        // every 1024 taken jumps (and before the SGPR count could overflow) the run
        // returns to the scheduler, which flushes counts and checks the limits
        if (pcs <= low) other = low;   // jumped back below every waiting lane
        if (--tick == 0 || (int32_t)sc < 0 || sc >= core_lim || pcs >= other) goto k_leave;
        I = code[pcs];
        continue;
      k_exit:
        sc += cnt8;
        xpost = post8;
        break;
      k_slow:
        slow = true;
      k_leave:
        xpc = pcs;
        tcode = 0;
        xadj = 0;
        break;
      }
#undef WB_FAST
#undef JUMP
#undef BRANCH
#undef JUMP_LANE
#undef TRAP
#undef FINISH
#undef EXIT_IF_TRAPPED
#undef TRAP_CHECK
#undef SLOW_OP
#undef SLOW_IF
#undef HOST_YIELD
#undef MEM_BYTES
#undef WB_GROW
      count += (uint64_t)(int64_t)(int32_t)sc + asc;
      cost += scost;
      if (tcode == 0) {
        pc = xpc;
        count += (int64_t)xadj;
      } else if (tcode == WB_TCODE_DONE) {
        status = WB_STATUS_OK;
      } else {
        status = tcode;
        count -= xpost;
      }
    }
    const uint64_t slowmask = __ballot(slow);
    [[maybe_unused]] const uint64_t ts2 = WB_NOW();
    WB_STAT_ADD(ST_CYC_FAST, ts2 - ts1);
    if (slowmask) WB_STAT_ADD(ST_SLOW, 1);
    if (slowmask && ((slowmask >> lane) & 1u)) {
      // ================================================================ slow step
      // One dispatch with fully per-lane semantics (the same step code, WB_FAST 0):
      // misaligned / out-of-bounds memory, traps, bulk memory ops, memory.grow,
      // call_indirect, leaving the entry function.
#define WB_FAST 0
#define TRAP(code) do { status = (code); add = (int32_t)cnt8 - (int32_t)post8; } while (0)
#define FINISH() (status = WB_STATUS_OK)
#define JUMP(t, tc) do { npc = (t); add += (tc); jtc = (tc); goto s_next; } while (0)
#define JUMP_LANE(t, tc) JUMP(t, tc)
#define BRANCH(c, t, tc) do { if (c) { npc = (t); add += (tc); jtc = (tc); } goto s_next; } while (0)
#define EXIT_IF_TRAPPED(t) ((void)0)
#define TRAP_CHECK() ((void)0)
#define SLOW_OP() ((void)0)
#define SLOW_IF(c) ((void)0)
#define HOST_YIELD(f, base) do { status = WB_ERR_HOST_CALL; ycall = (f); ybase = (base); } while (0)
#define MEM_BYTES ((uint64_t)slow_pages << 16)
      // memory.grow (dbc_step.inc): within the reserved pages or the wave's pool rows it
      // completes here; past them the lane parks for the host (hostcall.cpp grow service)
#define WB_GROW(cur, n, res) do { const uint32_t _np = (cur) + (n); \
    if (!PG) { pages = _np; res = (cur); } \
    else if (_np <= p.rpages || (_np - 1u - p.rpages < p.ptab_w && \
        p.ptab[(size_t)__builtin_amdgcn_readfirstlane(inst >> 6) * p.ptab_w + _np - 1u - p.rpages] != 0)) { \
      LS_PAGES_REF = _np; pages = min(_np, p.rpages); res = (cur); \
    } else { res = (n); HOST_YIELD(WB_GROW_CALL, C_); } } while (0)
      const uint32_t pcs = __builtin_amdgcn_readlane(pc, (uint32_t)__builtin_ctzll(slowmask));
      const uint32_t slow_pages = MEM_PAGES;   // the memory size (past the reserved layout too)
      const w4 I = code[pcs];
      const uint32_t w0 = I.x, w1 = I.y, w2 = I.z, w3 = I.w;
      const uint32_t op = w0 & 0x7FFFu;
      const uint32_t cnt8 = (w0 >> 16) & 0xFFu, post8 = (w0 >> 24) & 0x7Fu;
      const int32_t tcnt = (int32_t)(int16_t)(w2 >> 16);
      uint32_t npc = pcs + 1;
      int32_t add = (int32_t)cnt8, jtc = 0;
      const uint32_t coff = p.cost_off ? p.cost_off[pcs] : 0u;
      // engine.cpp:1616-1630: an instruction is counted, then its cost is added; past the
      // limit it fails with CostLimitExceeded before it executes. Here: the instructions
      // up to the main op first, then (if it did not trap) the ones after it, then a
      // taken branch's adjustment (gas_step in dbc_ops.h)
      // a call past the call stack's cells while the stack may still grow (KParams::
      // gs_grow; the reference's StackManager is a growing vector, stackmgr.h:44-47): the
      // lane parks at the call for the host to grow the stack (hostcall.cpp grow_stack) and
      // runs it again on resume -- counted and priced once, then
      if (p.gs_grow && (op == OP_CALL || op == OP_CALL_INDIRECT) &&
          gsp + ((w1 & 0xFFFFu) - p.global_cells) + 1 > p.gs_depth) {
        status = WB_ERR_HOST_CALL;
        ycall = WB_STACK_CALL;
        ybase = p.global_cells;
        add = 0;
        npc = pcs;
        goto s_done;
      }
      // a table.grow past its table's per-lane capacity, within the table's widen limit
      // (KParams::tg_grow; the reference's Refs vector grows up to the max, table.h:59-72):
      // the lane parks with the request n staged (ybase = its cell) for the host to widen
      // every lane's table (hostcall.cpp widen_tables) and runs the grow again on resume
      if (p.tg_grow && op == OP_TABLE_GROW) {
        const uint64_t want = (uint64_t)TSIZE(D_) + R32(B_);
        if (want > p.tabinfo[2u * D_ + 1u] && want <= p.tlimit[D_]) {
          status = WB_ERR_HOST_CALL;
          ycall = WB_TGROW_CALL | D_;
          ybase = B_;
          add = 0;
          npc = pcs;
          goto s_done;
        }
      }
      if (p.cost_off && gas_step(p.cost_pool + coff, 0, cnt8 - post8, p.cost_limit, cost, add)) {
        status = 0x03u;
        goto s_done;
      }
      // (memories past the first live only in the paged copy: a module with them runs the
      // PG kernels and takes that copy always)
      if (!PG || (!__ballot(pages >= p.rpages) && !p.n_xmem)) {
        switch (op) {
#define WB_XMEM_ON 0
#include "dbc_step.inc"
#undef WB_XMEM_ON
        }
      } else {
        // a lane of this group has grown past the reserved layout: the step's accesses go
        // through the paged view (pool rows too); the fast paths only ever see the
        // reserved layout (their bounds checks use min(pages, rpages)). A second copy of
        // the step, so that the paged addressing costs the common case nothing.
        const GMemP mem_pg{mem.p, mem.g, p.mem_words,
                           p.ptab ? p.ptab + (size_t)__builtin_amdgcn_readfirstlane(inst >> 6) * p.ptab_w : nullptr,
                           lane << p.mlog};
        const GMemP &mem = mem_pg;
        switch (op) {
#define WB_XMEM_ON 1
#include "dbc_step.inc"
#undef WB_XMEM_ON
        }
      }
    s_next:
      if (p.cost_off && (status == WB_STATUS_RUNNING || status == WB_STATUS_OK) &&
          gas_tail(p.cost_pool + coff, cnt8 - post8, cnt8, jtc,
                   jtc < 0 ? p.cost_pool + p.cost_off[npc] : nullptr, p.cost_else, p.cost_limit,
                   cost, add))
        status = 0x03u;
    s_done:
      count += (int64_t)add;
      pc = npc;
#undef WB_FAST
#undef JUMP
#undef BRANCH
#undef JUMP_LANE
#undef TRAP
#undef FINISH
#undef EXIT_IF_TRAPPED
#undef TRAP_CHECK
#undef SLOW_OP
#undef SLOW_IF
#undef HOST_YIELD
#undef MEM_BYTES
#undef WB_GROW
    }
    WB_STAT_ADD(ST_CYC_SLOW, WB_NOW() - ts2);
    // budget, wall clock, and the host's interrupt request (a core call returns at least
    // every 2^20 instructions) -- the reference's StopToken, checked on every branch, call
    // and return (helper.cpp:24-27,184-187, controlInstr.cpp:75-78). The flag is an
    // uncached system-scope read: at most one per 10 us of the wave's time (a round can be
    // a single slow-step instruction), so a request lands within 10 us + one round.
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    bool stop = false;
    if (now - tpoll >= 1000u) {
      tpoll = now;
      stop = __hip_atomic_load(p.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (status == WB_STATUS_RUNNING && (count >= p.max_steps || now - t0 > p.max_ticks || stop))
      status = WB_ERR_INTERRUPTED;
  }
#undef R32
#undef R64
#undef W32
#undef W64
#undef W128
#undef WLOOP
#undef GS_RD
#undef GS_WR
#undef GS_FAST
#undef GSF_BASE
#undef GS_PTR
#undef GS_CPTR
#ifdef WB_STATS
  if (p.stats && __lane_id() == (uint32_t)__builtin_ctzll(__ballot(1)))
    p.stats[(size_t)(inst >> 6) * 32u + ST_T1] = __builtin_amdgcn_s_memrealtime();
#endif
  if (active) {
    p.status[inst] = (uint8_t)status;
    p.counts[inst] = count;
    if (status == WB_ERR_HOST_CALL && fs) {   // park: the host loop takes over
      if (p.parked) *p.parked = 1u;
      LS(LS_RPC) = pc;
      LS(LS_GSP) = gsp;
      LS(LS_HBASE) = ybase;
      p.hcall[inst] = ycall;
      for (uint32_t c = p.global_cells; c < p.total_cells; c++) fs[(size_t)c << 6] = F.get(c);
      for (uint32_t k = 0; k < gsp && k < S_lds; k++) fs[(size_t)(p.total_cells + k) << 6] = stk[k << 6];
      for (uint32_t k = 0; k < p.hb_cells && ybase + k < p.total_cells; k++)
        p.hbuf[(size_t)inst * p.hb_cells + k] = F.get(ybase + k);
    }
    if (!PG) LS(LS_PAGES) = pages;   // (PG: memory.grow wrote it)
    LS(LS_DROPPED) = dropped;
    LS(LS_HWM) = hwm;
    LS(LS_COST) = (uint32_t)cost;
    LS(LS_COST + 1) = (uint32_t)(cost >> 32);
    for (uint32_t c = 0; c < p.global_cells; c++) LS(LS_GLOBALS + c) = F.get(c);
    if (p.is_start && status != WB_STATUS_OK) LS(LS_ISTATUS) = status;
  }
#undef LS
#undef WB_MARK
#undef ELEM_DROPPED
#undef SET_ELEM_DROPPED
#undef DATA_DROPPED
#undef SET_DATA_DROPPED
#undef MEM_PAGES
#undef LS_PAGES_REF
}

// General kernel: frames of any size in LDS (4 waves per block when they fit). VF: the
// threaded core keeps the frame in VGPRs (frames up to TC_VF_CELLS cells; 256 VGPRs).
// The wave of the batch a launch wave runs next: its own (blockIdx) when the launch has a
// wave per batch wave, else (persistent waves: more batch waves than the chip holds at
// once, C5's 4,096 at 2 per SIMD) the next one not yet taken -- a wave whose lanes finish
// early takes more work instead of leaving its SIMD idle until the slowest wave of its
// block ends. Every instance-state buffer is indexed by the batch wave, so which launch
// wave runs it does not matter. ~0: none left.
__device__ __forceinline__ uint32_t next_wave(const KParams &p, uint32_t &turn) {
  const uint32_t nwaves = (p.n + 63u) >> 6;
  if (!p.wave_ctr) return turn++ ? 0xFFFFFFFFu : (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  uint32_t w = 0;
  if ((threadIdx.x & 63u) == 0) w = __hip_atomic_fetch_add(p.wave_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  w = __builtin_amdgcn_readfirstlane(w);
  if (w >= nwaves) return 0xFFFFFFFFu;
  return p.wave_order ? __builtin_amdgcn_readfirstlane(p.wave_order[w]) : w;
}

// Instance state at instantiation (instantiate/module.cpp: memory of `min` pages, active
// data segments dropped, globals from their initialisers, no failure yet): LS slot `slot`.
struct StateInit {
  const uint32_t *global_init;
  uint32_t init_pages, init_dropped;
  uint64_t init_cost;
  uint32_t on;   // (mem init) reset the state too
};
__device__ __forceinline__ uint32_t state_word(uint32_t slot, const StateInit &st) {
  if (slot == LS_PAGES) return st.init_pages;
  if (slot == LS_DROPPED) return st.init_dropped;
  if (slot == LS_RPC) return 0xFFFFFFFFu;
  if (slot == LS_COST) return (uint32_t)st.init_cost;
  if (slot == LS_COST + 1) return (uint32_t)(st.init_cost >> 32);
  if (slot >= LS_GLOBALS) return st.global_init[slot - LS_GLOBALS];
  return 0;
}

// A Reset folded into the launch (KParams::rf_on; batch_api.cpp WasmEdge_BatchReset, 4-byte
// granules only): before its wave runs, each lane rewrites its own memory words below the
// wave's write mark (or the image) and its instance state -- wb_mem_init_kernel's
// write-mark path for one wave, with no kernel of its own. Every lane writes only its own
// column, so its later loads see the words in program order.
__device__ __forceinline__ void fused_reset(const KParams &p, uint32_t wave, uint32_t lane) {
  uint32_t *const lw = p.lstate + (size_t)wave * p.ls_slots * 64u + lane;
  uint32_t m = lw[(size_t)LS_HWM << 6];
  for (uint32_t o = 32; o; o >>= 1) m = max(m, (uint32_t)__shfl_xor(m, o, 64));
  const uint64_t hw = ((uint64_t)m + 3u) / 4u;
  uint32_t rows = (uint32_t)(hw < p.rf_init_words ? hw : p.rf_init_words);
  if (rows < p.rf_image_words && p.rf_image_words <= p.rf_init_words) rows = p.rf_image_words;
  uint32_t *const wm = p.mem + (size_t)wave * p.mem_words * 64u + lane;
  for (uint32_t w = 0; w < rows; w++) wm[(size_t)w << 6] = w < p.rf_image_words ? p.rf_image[w] : 0u;
  // (state_word's words, from the kernel arguments: no StateInit on the stack)
  for (uint32_t slot = 0; slot < p.ls_slots; slot++)
    lw[(size_t)slot << 6] = slot == LS_PAGES ? p.rf_init_pages : slot == LS_DROPPED ? p.rf_init_dropped
                          : slot == LS_RPC ? 0xFFFFFFFFu : slot == LS_COST ? (uint32_t)p.rf_init_cost
                          : slot == LS_COST + 1 ? (uint32_t)(p.rf_init_cost >> 32)
                          : slot >= LS_GLOBALS ? p.rf_global_init[slot - LS_GLOBALS] : 0u;
}

template <bool VF, bool PG>
__device__ __forceinline__ void exec_body(const KParams &p) {
  extern __shared__ uint32_t lds[];
  const uint32_t lane = threadIdx.x & 63u, wib = threadIdx.x >> 6;
  LdsFrame F{(lds_u32 *)(lds + ((wib * p.total_cells) << 6) + lane)};
  // LDS call-stack slots of this wave follow the frames of all the block's waves
  lds_u32 *const stk = (lds_u32 *)(lds + ((((blockDim.x >> 6) * p.total_cells) + wib * p.gs_lds) << 6) + lane);
  uint32_t turn = 0;
  for (uint32_t wave; (wave = next_wave(p, turn)) != 0xFFFFFFFFu;) {
    const uint32_t inst = wave * 64u + lane;
    if (p.rf_on && wave < ((p.n + 63u) >> 6)) fused_reset(p, wave, lane);   // (batch waves only)
    const uint64_t ws = p.wave_ticks ? __builtin_amdgcn_s_memrealtime() : 0;
    interp<VF, PG>(p, F, inst, p.gstack + (size_t)wave * p.gs_depth * 64u + lane,
               GMem{p.mem + (size_t)wave * p.mem_words * 64u + (lane << p.mlog), p.mlog},
               p.lstate + (size_t)wave * p.ls_slots * 64u + lane,
               p.fsave ? p.fsave + (size_t)wave * (p.total_cells + p.gs_lds) * 64u + lane : nullptr, stk);
    if (p.wave_ticks && lane == 0)
      p.wave_ticks[wave] = (uint32_t)min(__builtin_amdgcn_s_memrealtime() - ws, 0xFFFFFFFFull);
  }
}

extern "C" __global__ void __launch_bounds__(256, 4) wb_exec_kernel(const KParams p) {
  exec_body<false, false>(p);
}
extern "C" __global__ void __launch_bounds__(256, 4) wb_exec_pg_kernel(const KParams p) {
  exec_body<false, true>(p);
}
// HBM frames: LDS holds only the waves' call-stack slots
template <bool PG>
__device__ __forceinline__ void exec_hbm_body(const KParams &p) {
  extern __shared__ uint32_t lds[];
  const uint32_t lane = threadIdx.x & 63u, wib = threadIdx.x >> 6;
  lds_u32 *const stk = (lds_u32 *)(lds + ((wib * p.gs_lds) << 6) + lane);
  uint32_t turn = 0;
  for (uint32_t wave; (wave = next_wave(p, turn)) != 0xFFFFFFFFu;) {
    const uint32_t inst = wave * 64u + lane;
    if (p.rf_on && wave < ((p.n + 63u) >> 6)) fused_reset(p, wave, lane);   // (batch waves only)
    const uint64_t ws = p.wave_ticks ? __builtin_amdgcn_s_memrealtime() : 0;
    HbmFrame F{p.hframe + (size_t)wave * p.total_cells * 64u + lane};
    interp<false, PG>(p, F, inst, p.gstack + (size_t)wave * p.gs_depth * 64u + lane,
                  GMem{p.mem + (size_t)wave * p.mem_words * 64u + (lane << p.mlog), p.mlog},
                  p.lstate + (size_t)wave * p.ls_slots * 64u + lane,
                  p.fsave ? p.fsave + (size_t)wave * (p.total_cells + p.gs_lds) * 64u + lane : nullptr, stk);
    // (the longest-first order of the next launch reads these, as for the other frames)
    if (p.wave_ticks && lane == 0)
      p.wave_ticks[wave] = (uint32_t)min(__builtin_amdgcn_s_memrealtime() - ws, 0xFFFFFFFFull);
  }
}
extern "C" __global__ void __launch_bounds__(256) wb_exec_hbm_kernel(const KParams p) {
  exec_hbm_body<false>(p);
}
extern "C" __global__ void __launch_bounds__(256) wb_exec_hbm_pg_kernel(const KParams p) {
  exec_hbm_body<true>(p);
}
extern "C" __global__ void __launch_bounds__(256, 2) wb_exec_vf_kernel(const KParams p) {
  exec_body<true, false>(p);
}
extern "C" __global__ void __launch_bounds__(256, 2) wb_exec_vf_pg_kernel(const KParams p) {
  exec_body<true, true>(p);
}

// ======================================================================= helpers
// Instantiation image broadcast (instantiate/memory.cpp + data.cpp): every lane's
// pages [0, init_pages) = the module image (data segments), the rest of those pages zero.
// Block b covers rows [c*1024, (c+1)*1024) of wave b / chunks (a row = one word of the 64
// lanes). Unless `full`, only rows below the wave's highest write mark (LS_HWM, bytes)
// or the image are rewritten: memory above it was zeroed by the previous instantiation
// and never written since (the kernel's every store path raises the mark), the way the
// reference's fresh MAP_ANONYMOUS pages are zero without being written. `ls` = nullptr:
// always full (per-lane table images).
// `init_words` = the rows this covers: the whole reserved layout (rpages), so that pages a
// lane grows into later read zero without memory.grow writing them; pool rows are zeroed
// by the host (batch_api.cpp pool_reset).
// (write-mark path) with st.on set, the wave's instance state is reset too, after
// its mark was read: one launch per Reset instead of two
extern "C" __global__ void __launch_bounds__(256)
wb_mem_init_kernel(uint32_t *mem, const uint32_t *image, uint32_t image_words,
                   uint32_t init_words, uint32_t mem_words, uint32_t nwaves,
                   uint32_t *ls, uint32_t ls_slots, uint32_t full, uint32_t g, StateInit st) {
  const uint32_t chunks = (init_words + 1023u) / 1024u;
  if (!full && ls) {
    // a Reset after a run: 64 threads per batch wave (4 per block) read the wave's write
    // marks once (a shuffle max) and rewrite the rows below the highest (usually a few; the
    // mark is per lane, the rows per wave)
    const uint32_t lane = threadIdx.x & 63u;
    for (size_t wave = (size_t)blockIdx.x * 4u + (threadIdx.x >> 6); wave < nwaves;
         wave += (size_t)gridDim.x * 4u) {
      uint32_t m = ls[((size_t)wave * ls_slots + LS_HWM) * 64u + lane];
      for (uint32_t o = 32; o; o >>= 1) m = max(m, (uint32_t)__shfl_xor(m, o, 64));
      const uint64_t hw = ((uint64_t)m + 3u) / 4u;
      uint32_t rows = (uint32_t)(hw < init_words ? hw : init_words);
      if (rows < image_words && image_words <= init_words) rows = image_words;
      const uint32_t gm = (1u << g) - 1u;
      rows = (rows + gm) & ~gm;
      if (rows > init_words) rows = init_words;
      uint32_t *wm = mem + wave * mem_words * (size_t)64u;
      for (size_t i = lane; i < (size_t)rows * 64u; i += 64u) {
        const uint32_t word = (uint32_t)(((i >> (6 + g)) << g) | (i & ((1u << g) - 1u)));
        wm[i] = word < image_words ? image[word] : 0u;
      }
      if (st.on) {   // (after every lane's mark was read: the shuffle)
        uint32_t *lw = ls + (size_t)wave * ls_slots * 64u;
        for (uint32_t i = lane; i < ls_slots * 64u; i += 64u) lw[i] = state_word(i >> 6, st);
      }
    }
    return;
  }
  for (size_t b = blockIdx.x; b < (size_t)nwaves * chunks; b += gridDim.x) {
    const size_t wave = b / chunks;
    const uint32_t r0 = (uint32_t)(b - wave * chunks) * 1024u;
    const uint32_t rows = init_words;
    const uint32_t r1 = r0 + 1024u < rows ? r0 + 1024u : rows;
    if (r1 <= r0) continue;
    uint32_t *wm = mem + wave * mem_words * (size_t)64u;
    // size_t: rows past 2^26 (initial memories over 4096 pages) must not wrap
    for (size_t i = (size_t)r0 * 64u + threadIdx.x; i < (size_t)r1 * 64u; i += blockDim.x) {
      // linear index -> word: granule i >> (6 + g), word (i & (2^g - 1)) within it
      const uint32_t word = (uint32_t)(((i >> (6 + g)) << g) | (i & ((1u << g) - 1u)));
      wm[i] = word < image_words ? image[word] : 0u;
    }
  }
}

// Instance state at instantiation, every wave (a Reset without the write-mark path).
extern "C" __global__ void __launch_bounds__(256)
wb_state_init_kernel(uint32_t *ls, uint32_t ls_slots, uint32_t nwaves, StateInit st) {
  const size_t total = (size_t)nwaves * ls_slots * 64u;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x)
    ls[i] = state_word((uint32_t)((i >> 6) % ls_slots), st);
}

// Memory hash: sum over u64 words of fmix64(w ^ (i*K1 + K2)), ^ fmix64(pages+K3).
// The sum commutes, so the words are spread over the grid: block (wave, c) adds the terms
// of u64 words [c*8192, (c+1)*8192) -- page c -- of its wave's 64 lanes into hashes[]
// (zeroed first), and wb_mem_hash_fin_kernel XORs the page-count term in.
//
// Page c of a wave's 64 lanes is ONE contiguous 4 MiB region in the interleaved layout
// (the reserved layout, or the wave's pool row for a page past it), so the block streams
// it front to back in 16-byte pieces -- a wave's load is 1 KiB contiguous, the access the
// guide calibrates FETCH_SIZE on (MI355X_MICROARCH.md "HBM": 16 B per lane). Which lane
// and word a piece holds follows from the granule of 2^g words:
//   g >= 2: 4 consecutive words of one lane (a granule is 2^(g-2) pieces);
//   g == 1: a u64 word of each of two adjacent lanes;
//   g == 0: a lane's u64 word is two words a 64-word row apart, so a thread reads the same
//           piece of two consecutive rows (a u64 word of each of 4 lanes).
// A thread serves fixed lanes (one or two; four at g == 0) over its whole loop, so its
// terms add up in registers, then per lane in LDS, then one global atomic per lane.
typedef uint32_t wb_u32x4 __attribute__((ext_vector_type(4)));
#define WB_HK(x, i) fmix64((x) ^ ((uint64_t)(i) * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull))
extern "C" __global__ void __launch_bounds__(256)
wb_mem_hash_kernel(uint32_t *mem, const uint32_t *ls, uint32_t ls_slots,
                   uint64_t *hashes, uint32_t mem_words, uint32_t n, uint32_t g,
                   const uint64_t *ptab, uint32_t ptab_w) {
  const uint32_t wave = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  __shared__ unsigned long long acc[64];
  __shared__ uint32_t ok[64];
  __shared__ uint32_t any;
  if (t == 0) any = 0;
  __syncthreads();
  if (t < 64) {
    const uint32_t inst = wave * 64u + t;
    ok[t] = inst < n && c < ls[((size_t)wave * ls_slots + LS_PAGES) * 64u + t];
    acc[t] = 0;
    if (ok[t]) any = 1;   // (benign race: every writer writes 1)
  }
  __syncthreads();
  if (!any) return;
  const uint32_t rp = mem_words >> 14;   // pages in the reserved layout
  const wb_u32x4 *src;
  if (c < rp) {
    src = (const wb_u32x4 *)(mem + ((size_t)wave * mem_words + ((size_t)c << 14)) * 64u);
  } else {
    const uint64_t row = ptab ? ptab[(size_t)wave * ptab_w + (c - rp)] : 0;
    if (!row) return;   // (no lane of the wave is that large: `any` was 0)
    src = (const wb_u32x4 *)(uintptr_t)row;
  }
  const uint64_t i0 = (uint64_t)c << 13;   // the page's first u64 word
  uint64_t h[4] = {0, 0, 0, 0};
  uint32_t ln[4];
  if (g >= 2) {
    const uint32_t s = g - 2;
    ln[0] = (t >> s) & 63u;
    ln[1] = ((t >> s) + (256u >> s)) & 63u;   // (== ln[0] unless s == 3)
    const bool v0 = ok[ln[0]], v1 = ok[ln[1]];
#pragma unroll 4
    for (uint32_t k = 0; k < 1024u; k++) {
      const uint32_t j = t + 256u * k;
      if (!((k & 1u) ? v1 : v0)) continue;
      const wb_u32x4 x = __builtin_nontemporal_load(&src[j]);
      const uint64_t i = i0 + ((((uint64_t)(j >> (s + 6)) << g) + ((j & ((1u << s) - 1u)) << 2)) >> 1);
      h[k & 1u] += WB_HK((uint64_t)x.x | ((uint64_t)x.y << 32), i) + WB_HK((uint64_t)x.z | ((uint64_t)x.w << 32), i + 1);
    }
    if (s == 3) {
      if (v0) atomicAdd(&acc[ln[0]], (unsigned long long)h[0]);
      if (v1) atomicAdd(&acc[ln[1]], (unsigned long long)h[1]);
    } else if (v0) {
      atomicAdd(&acc[ln[0]], (unsigned long long)(h[0] + h[1]));
    }
  } else if (g == 1) {
    ln[0] = (2u * t) & 63u;
    ln[1] = ln[0] + 1u;
    const bool v0 = ok[ln[0]], v1 = ok[ln[1]];
    if (v0 || v1) {
#pragma unroll 4
      for (uint32_t k = 0; k < 1024u; k++) {
        const uint32_t j = t + 256u * k;
        const wb_u32x4 x = __builtin_nontemporal_load(&src[j]);
        const uint64_t i = i0 + (j >> 5);
        h[0] += WB_HK((uint64_t)x.x | ((uint64_t)x.y << 32), i);
        h[1] += WB_HK((uint64_t)x.z | ((uint64_t)x.w << 32), i);
      }
      if (v0) atomicAdd(&acc[ln[0]], (unsigned long long)h[0]);
      if (v1) atomicAdd(&acc[ln[1]], (unsigned long long)h[1]);
    }
  } else {
    const uint32_t m = t & 15u;   // piece of the 64-word row: lanes 4m .. 4m+3
    bool v[4];
    for (uint32_t q = 0; q < 4; q++) {
      ln[q] = 4u * m + q;
      v[q] = ok[ln[q]];
    }
    if (v[0] || v[1] || v[2] || v[3]) {
#pragma unroll 4
      for (uint32_t k = 0; k < 512u; k++) {
        const uint32_t r = (t >> 4) + 16u * k;   // u64 word r: rows 2r and 2r+1
        const wb_u32x4 lo = __builtin_nontemporal_load(&src[(2u * r) * 16u + m]);
        const wb_u32x4 hi = __builtin_nontemporal_load(&src[(2u * r + 1u) * 16u + m]);
        const uint64_t i = i0 + r;
        h[0] += WB_HK((uint64_t)lo.x | ((uint64_t)hi.x << 32), i);
        h[1] += WB_HK((uint64_t)lo.y | ((uint64_t)hi.y << 32), i);
        h[2] += WB_HK((uint64_t)lo.z | ((uint64_t)hi.z << 32), i);
        h[3] += WB_HK((uint64_t)lo.w | ((uint64_t)hi.w << 32), i);
      }
      for (uint32_t q = 0; q < 4; q++)
        if (v[q]) atomicAdd(&acc[ln[q]], (unsigned long long)h[q]);
    }
  }
  __syncthreads();
  if (t < 64 && ok[t]) atomicAdd((unsigned long long *)&hashes[wave * 64u + t], acc[t]);
}
#undef WB_HK
extern "C" __global__ void __launch_bounds__(256)
wb_mem_hash_fin_kernel(const uint32_t *ls, uint32_t ls_slots, uint64_t *hashes, uint32_t n) {
  const uint32_t inst = blockIdx.x * blockDim.x + threadIdx.x;
  if (inst >= n) return;
  const uint32_t pages = ls[((size_t)(inst >> 6) * ls_slots + LS_PAGES) * 64u + (inst & 63u)];
  hashes[inst] ^= fmix64((uint64_t)pages + 0x1234567ull);
}

// Longest-first order of the batch waves for the next persistent launch (KParams::
// wave_order), from this launch's per-wave run times: a counting sort over 1024 buckets of
// [0, max] (descending), in one block -- on the device, so no host round trip sits between
// launches. Within a bucket the order is whatever the atomics give (scheduling only).
extern "C" __global__ void __launch_bounds__(1024)
wb_wave_order_kernel(const uint32_t *ticks, uint32_t *order, uint32_t nwaves, uint32_t *wave_ctr) {
  __shared__ uint32_t cnt[1024];
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t mx;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  cnt[t] = 0;
  if (t == 0) {
    mx = 0;
    *wave_ctr = 0;   // the next persistent launch starts from batch wave 0 (no memset)
  }
  __syncthreads();
  for (uint32_t w = t; w < nwaves; w += 1024) atomicMax(&mx, ticks[w]);
  __syncthreads();
  const uint64_t span = (uint64_t)mx + 1;
  for (uint32_t w = t; w < nwaves; w += 1024)
    atomicAdd(&cnt[1023u - (uint32_t)((uint64_t)ticks[w] * 1024u / span)], 1u);
  __syncthreads();
  // exclusive prefix sum over the buckets, heaviest first: a shuffle scan per wave, then
  // the 16 wave totals
  const uint32_t c = cnt[t];
  uint32_t x = c;
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  uint32_t off = 0;
  for (uint32_t i = 0; i < wv; i++) off += wsum[i];
  cnt[t] = off + x - c;
  __syncthreads();
  for (uint32_t w = t; w < nwaves; w += 1024)
    order[atomicAdd(&cnt[1023u - (uint32_t)((uint64_t)ticks[w] * 1024u / span)], 1u)] = w;
}

// ======================================================================= launchers
extern "C" hipError_t wb_launch_wave_order(const uint32_t *ticks, uint32_t *order, uint32_t nwaves,
                                           uint32_t *wave_ctr, hipStream_t s) {
  hipLaunchKernelGGL(wb_wave_order_kernel, dim3(1), dim3(1024), 0, s, ticks, order, nwaves, wave_ctr);
  return hipGetLastError();
}
// (host stubs live in this translation unit; the C-ABI layer calls these)
// the kernel for a launch: frames in HBM / LDS / VGPRs, and paged (PG) or not
static const void *exec_kernel(int vframe, int hbm, int paged) {
  if (hbm) return paged ? reinterpret_cast<const void *>(&wb_exec_hbm_pg_kernel)
                        : reinterpret_cast<const void *>(&wb_exec_hbm_kernel);
  if (vframe) return paged ? reinterpret_cast<const void *>(&wb_exec_vf_pg_kernel)
                           : reinterpret_cast<const void *>(&wb_exec_vf_kernel);
  return paged ? reinterpret_cast<const void *>(&wb_exec_pg_kernel)
               : reinterpret_cast<const void *>(&wb_exec_kernel);
}
// The 160 KiB dynamic-LDS attribute of every exec kernel variant, once per device: HIP keeps
// function attributes per device, and a multi-device batch (multi.cpp) launches on several.
static void exec_attrs() {
  static std::mutex mu;
  static std::vector<bool> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return;
  std::lock_guard<std::mutex> g(mu);
  if (size_t(dev) < done.size() && done[dev]) return;
  if (done.size() <= size_t(dev)) done.resize(size_t(dev) + 1, false);
  for (int k = 0; k < 8; k++)
    (void)hipFuncSetAttribute(exec_kernel(k & 1, k >> 1 & 1, k >> 2 & 1),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  done[dev] = true;
}
extern "C" hipError_t wb_launch_exec(const KParams *p, uint32_t blocks, uint32_t threads,
                                     size_t lds_bytes, int vframe, hipStream_t s) {
  exec_attrs();
  const void *k = exec_kernel(vframe, p->hframe != nullptr, p->grow_host != 0 || p->n_xmem != 0);
  void *args[] = {const_cast<KParams *>(p)};
  return hipLaunchKernel(k, dim3(blocks), dim3(threads), args, lds_bytes, s);
}
// Blocks of the exec kernel the whole device holds at once (persistent waves, KParams::
// wave_ctr): resident blocks per CU at this block size and LDS share x CUs; 0 on failure.
extern "C" uint32_t wb_exec_capacity(int vframe, int hbm, int paged, uint32_t threads, size_t lds_bytes) {
  int per_cu = 0, cus = 0, dev = 0;
  exec_attrs();
  const void *k = exec_kernel(vframe, hbm, paged);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, int(threads), lds_bytes) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return uint32_t(per_cu > 0 ? per_cu : 0) * uint32_t(cus > 0 ? cus : 0);
}
extern "C" hipError_t wb_launch_mem_init(uint32_t *mem, const uint32_t *image,
                                         uint32_t image_words, uint32_t init_words,
                                         uint32_t mem_words, uint32_t nwaves,
                                         uint32_t *ls, uint32_t ls_slots, uint32_t full,
                                         uint32_t g, uint32_t fuse_state, const uint32_t *global_init,
                                         uint32_t init_pages, uint32_t init_dropped,
                                         uint64_t init_cost, hipStream_t s) {
  const size_t total = (size_t)nwaves * ((init_words + 1023u) / 1024u);
  if (total == 0) return hipSuccess;
  // full (re)initialisation: a block per 1024 rows of a wave; after a run: 64 threads per
  // wave (the kernel's write-mark path, which also resets the instance state when
  // fuse_state is set)
  const size_t blocks = (!full && ls) ? (nwaves + 3u) / 4u : (total < 262144 ? total : 262144);
  const StateInit st{global_init, init_pages, init_dropped, init_cost, (!full && ls && fuse_state) ? 1u : 0u};
  hipLaunchKernelGGL(wb_mem_init_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, mem, image,
                     image_words, init_words, mem_words, nwaves, ls, ls_slots, full, g, st);
  return hipGetLastError();
}
extern "C" hipError_t wb_launch_mem_hash(uint32_t *mem, const uint32_t *ls,
                                         uint32_t ls_slots, uint64_t *hashes,
                                         uint32_t mem_words, uint32_t n, uint32_t g,
                                         const uint64_t *ptab, uint32_t ptab_w, uint32_t max_pages,
                                         hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(hashes, 0, size_t(n) * 8, s);
  if (e != hipSuccess) return e;
  if (max_pages)
    hipLaunchKernelGGL(wb_mem_hash_kernel, dim3((n + 63) / 64, max_pages), dim3(256), 0, s, mem, ls,
                       ls_slots, hashes, mem_words, n, g, ptab, ptab_w);
  hipLaunchKernelGGL(wb_mem_hash_fin_kernel, dim3((n + 255) / 256), dim3(256), 0, s, ls, ls_slots,
                     hashes, n);
  return hipGetLastError();
}
extern "C" hipError_t wb_launch_state_init(uint32_t *ls, uint32_t ls_slots, uint32_t nwaves,
                                           const uint32_t *global_init, uint32_t init_pages,
                                           uint32_t init_dropped, uint64_t init_cost, hipStream_t s) {
  const size_t total = (size_t)nwaves * ls_slots * 64u;
  size_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  const StateInit st{global_init, init_pages, init_dropped, init_cost, 1u};
  hipLaunchKernelGGL(wb_state_init_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, ls, ls_slots,
                     nwaves, st);
  return hipGetLastError();
}
