// tc.h -- threaded code (TInstr) for the hand-written dispatch core (gen_tc.py).
//
// One TInstr per DBC instruction (same pc), 32 bytes = one s_load_dwordx8:
//   w0 handler byte offset within a bank (slot * TC_SLOT_BYTES; 0 = no handler)
//   w1 a, w2 b, w5 d: LDS byte offsets (cell * 256) of the operands the core reads
//      ahead for every instruction (always valid cells); the V-frame blob takes cell
//      indices instead (w3, w7 cells alike)
//   w3 c: destination cell offset; compare-and-branch *_I: the sign-extended imm16
//   w4 immediate / memarg offset; branches: target pc * 32
//   w6 wasm instructions retired when the instruction falls through
//   w7 branches: instructions retired when taken (cnt + tcnt); loads/stores:
//      offset + bytes - 1; const64: the high word
#pragma once
#include <cstdint>
#include <vector>

#include "dbc.h"

#define DBC_HOT 0x8000u   // w0 bit 15 of a DBC instruction: the core has a handler

struct TInstr {
  uint32_t w[8];
};

namespace wb {
struct Program;
// Build the TInstr array for P (size = code + 2 padding entries for the core's
// successor prefetch) and mark DBC_HOT on the device copy `code` of P.code. vframe:
// fields for the V-frame blob (frame cells in VGPRs; needs total cells <= TC_VF_CELLS).
// run_start (optional): pcs where a compiled run will begin (jit.h); no fused tuple
// handler covers one of them past its first instruction.
// xinfo / xlog: (memories past the first) the context's word offsets and granule
// (batch_ctx.h xinfo_h, xlog) for the V blob's XLD / XST handlers; without them those
// instructions have no handler (the C++ step runs them).
std::vector<TInstr> build_threaded(const Program &P, std::vector<DInstr> &code, bool vframe,
                                   const std::vector<uint8_t> *run_start = nullptr,
                                   const std::vector<uint32_t> *xinfo = nullptr, uint32_t xlog = 0);
// Jump targets and resume points of P (index pc; size code + 1): branch/br_table/call
// targets, the instruction after every call, function entries and bodies.
std::vector<uint8_t> jump_targets(const Program &P);
}  // namespace wb
