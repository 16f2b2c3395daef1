// jit.h -- per-module compiled runs for the V-frame threaded core.
//
// The threaded core (gen_tc.py) spends most of a dispatch on the dispatch itself: the
// s_load of the next TInstr, the s_setpc, the GPR-index moves that name frame cells by
// an SGPR field. For a straight-line run of instructions (no jump target inside, every
// instruction one the compiler below knows) all of that is known when the module is
// loaded, so jit.cpp writes the run as plain CDNA4 assembly over the frame VGPRs
// (cell i = v[128 + i], the V-frame blob's layout), compiles it with hiprtc into a code
// object of its own and patches the run's first TInstr to the core's JIT slot, which
// jumps there. The run's code retires the run and dispatches the instruction after it
// through the core's bank-A handlers, or leaves through the core's exit stubs (slot 0)
// when a memory access fails its bounds or alignment check (the C++ step then executes
// that instruction, exactly as when a handler leaves). Results never depend on it:
// WB_JIT=0 turns it off, and the parity tests run both ways.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "tc.h"

namespace wb {
struct Program;

struct JitRun {
  uint32_t pc;    // first instruction
  uint32_t len;   // instructions
  uint32_t cnt;   // wasm instructions retired by the whole run
};

// Runs worth compiling: maximal straight-line stretches of compilable instructions with
// no jump target past their first, at least kMinRun long. `tc`: build_threaded's array
// (an instruction without a handler there is never compiled).
// simt: (KParams::simt) lone conditional branches and br_table end runs too, so that
// their splits stay in the core. trip: runs for trip mode (below): any length, lone jumps
// too (a lane at a pc outside every run waits outside the trips).
std::vector<JitRun> jit_runs(const Program &P, const std::vector<TInstr> &tc, bool simt = false,
                             bool trip = false);

// Gas prices of a metered context (batch_ctx.h cost_off_h / cost_pool_h): per DBC
// instruction its cost list's prefix sums. A compiled run checks at entry that every lane
// can pay its most expensive exit (else it leaves to the exact per-lane step) and adds
// the exact price of the exit it takes (the same sums as gas_step / gas_tail).
struct JitCost {
  const std::vector<uint32_t> *off;
  const std::vector<uint64_t> *pool;
  uint64_t c_else;   // price of an `else` a taken if-false branch retires
  uint64_t full(const Program &P, uint32_t pc) const;
  // a taken branch's correction (tcnt = jtc) landing at pc `to`
  int64_t taken(uint32_t to, int32_t jtc) const;
};

// The hiprtc source: one kernel, wbjit_addrs(uint64_t *out), that writes the address of
// run k's code to out[k]; the runs' code sits inside it behind branches. glog: linear-
// memory granule = 4 << glog bytes (batch_ctx.h lane_word). cost: metered contexts.
// simt: lanes that part ways (a split branch or return, reaching a waiting lane) stay in
// the core and are scheduled there (Lsched, KParams::simt); not with cost.
// Trip mode visits every run twice per trip: modules with more runs keep SIMT scheduling.
constexpr size_t kTripMaxRuns = 96;
// trip: (with simt, not with cost) trip mode instead of per-group runs: every lane of the
// wave at a run start runs that run in each trip, all of them together (jit.cpp "Trip
// mode"); for modules whose lanes part ways on loaded data.
// xinfo: (modules with memories past the first) the context's xinfo_h -- memory k's word
// offset in a lane's block at [2 (k - 1)] -- for the compiled XLD / XST (jit.cpp
// emit_xmem, which address the wave's block through s[98:99], set by the kernel at every
// core call); without it such a module gets no source. xlog: their granule (KParams::xlog).
// mem_pages: the first memory's page limit (the context's mem_max_pages): trip stages of a
// memory below 1,000 pages compute granule addresses in 32 bits (jit.cpp granule_addr).
std::string jit_source(const Program &P, const std::vector<JitRun> &runs, uint32_t glog,
                       const JitCost *cost = nullptr, bool simt = false, bool trip = false,
                       const std::vector<uint32_t> *xinfo = nullptr, uint32_t xlog = 0,
                       uint32_t mem_pages = 65536);

// Whether trip mode pays for a module whose memory addresses do not depend on per-instance
// data (Program::divergent_mem picks it for those): lanes part ways inside a loop on every
// trip round it -- a conditional branch whose two successors, or a br_table with two
// entries, stay in the innermost loop around it (C4's br_table state machine: 7.7e11
// against 6.1e11 instr/s on SIMT) -- and the module makes no calls (recursion's
// call/return transitions are cheaper under SIMT scheduling: C1 0.82x with trips).
// Loops whose lanes leave one by one (C5's escape loop: 0.59x with trips) do not qualify.
bool trips_pay(const Program &P);

// Compile `src` for gfx950 (hiprtc). Returns "" and the code object, or an error.
std::string jit_compile(const std::string &src, std::vector<char> *code, const std::string &arch = "gfx950");

// Compile (cached per device and source), load on the current device and read back the
// runs' code addresses. Returns "" or an error.
std::string jit_load(const std::string &src, size_t nruns, int device, std::vector<uint64_t> *addr);

// Point each run's first TInstr at its code (the core's JIT slot).
void jit_patch(std::vector<TInstr> &tc, const std::vector<JitRun> &runs, const std::vector<uint64_t> &addr);
}  // namespace wb
