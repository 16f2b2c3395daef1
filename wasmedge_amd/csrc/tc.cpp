// tc.cpp -- host translation of the DBC program into threaded code for the gfx950
// dispatch core (gen_tc.py / tc_blob.inc). Field layout: tc.h.
#include "tc.h"

#include <cstdlib>

#include "frontend.h"
#include "tc_slots.h"

namespace wb {

static uint32_t mem_bytes(uint16_t op) {
  switch (op) {
    case OP_LD8S32: case OP_LD8U32: case OP_LD8S64: case OP_LD8U64: case OP_ST8: return 1;
    case OP_LD16S32: case OP_LD16U32: case OP_LD16S64: case OP_LD16U64: case OP_ST16: return 2;
    case OP_LD32: case OP_LD32S64: case OP_LD32U64: case OP_ST32: return 4;
    case OP_LD64: case OP_ST64: return 8;
    default: return 0;
  }
}

static bool is_branch(uint16_t op) {
  return op == OP_JMP || op == OP_BR_IF || op == OP_BR_UNLESS ||
         (op >= OP_BR_EQ && op <= OP_BR_GE_U_I);
}

std::vector<uint8_t> jump_targets(const Program &P) {
  const size_t n = P.code.size();
  std::vector<uint8_t> target(n + 1, 0);
  for (size_t pc = 0; pc < n; pc++) {
    const DInstr &I = P.code[pc];
    const uint16_t op = uint16_t(I.w0 & 0x7FFFu);
    if ((is_branch(op) || op == OP_BR_IF_MOV1 || op == OP_BR_IF_MOV2 || op == OP_CALL || op == OP_TAIL_CALL) &&
        I.w3 < n)
      target[I.w3] = 1;
    if (op == OP_CALL || op == OP_CALL_INDIRECT || op == OP_HOST_CALL) target[pc + 1] = 1;
  }
  for (size_t k = 0; k + 1 < P.brtab.size(); k += 2)
    if (P.brtab[k] < n) target[P.brtab[k]] = 1;
  for (const auto &f : P.funcs)
    if (!f.imported) { target[f.entry_pc] = 1; target[f.body_pc] = 1; }
  return target;
}

// the V blob's handler of an extra memory's access (XLD / XST with the memory-0 op `mop`)
static int tc_xslot(uint16_t op, uint16_t mop) {
  if (op == OP_XLD) {
    switch (mop) {
      case OP_LD32: return TC_SLOT_XLD_LD32;
      case OP_LD8U32: return TC_SLOT_XLD_LD8U32;
      case OP_LD8S32: return TC_SLOT_XLD_LD8S32;
      case OP_LD16U32: return TC_SLOT_XLD_LD16U32;
      case OP_LD16S32: return TC_SLOT_XLD_LD16S32;
      case OP_LD32U64: return TC_SLOT_XLD_LD32U64;
      case OP_LD32S64: return TC_SLOT_XLD_LD32S64;
      case OP_LD8U64: return TC_SLOT_XLD_LD8U64;
      case OP_LD8S64: return TC_SLOT_XLD_LD8S64;
      case OP_LD16U64: return TC_SLOT_XLD_LD16U64;
      case OP_LD16S64: return TC_SLOT_XLD_LD16S64;
      case OP_LD64: return TC_SLOT_XLD_LD64;
      default: return 0;
    }
  }
  switch (mop) {
    case OP_ST8: return TC_SLOT_XST_ST8;
    case OP_ST16: return TC_SLOT_XST_ST16;
    case OP_ST32: return TC_SLOT_XST_ST32;
    case OP_ST64: return TC_SLOT_XST_ST64;
    default: return 0;
  }
}

std::vector<TInstr> build_threaded(const Program &P, std::vector<DInstr> &code, bool vframe,
                                   const std::vector<uint8_t> *run_start,
                                   const std::vector<uint32_t> *xinfo, uint32_t xlog) {
  const uint32_t T = P.total_cells();
  // operand fields: LDS byte offsets (cell * 256) for the LDS-frame blob, cell indices
  // (= VGPR index past v128) for the V-frame blob
  const uint32_t unit = vframe ? 1u : 256u;
  auto off = [T, unit](uint32_t cell) { return cell < T ? cell * unit : 0u; };
  std::vector<TInstr> tc(P.code.size() + 2, TInstr{{0, 0, 0, 0, 0, 0, 0, 0}});
  const char *tte = getenv("WB_TC_TAIL");
  const bool tail_off = tte && tte[0] == '0';
  for (size_t pc = 0; pc < P.code.size(); pc++) {
    const DInstr &I = P.code[pc];
    const uint16_t op = uint16_t(I.w0 & 0x7FFFu);
    const uint32_t a = I.w1 & 0xFFFFu, b = I.w1 >> 16, c = I.w2 & 0xFFFFu, d = I.w2 >> 16;
    const uint32_t imm = I.w3, cnt = (I.w0 >> 16) & 0xFFu;
    int slot = tc_slot(op);
    // (memories past the first: V blob, with the context's layout; gen_tc.py xmem_addr)
    const bool xop = (op == OP_XLD || op == OP_XST) && vframe && xinfo;
    const uint32_t xk = op == OP_XLD ? b : c;
    if (xop && xk >= 1 && xk <= P.xmems.size() && size_t(2 * xk) <= xinfo->size() &&
        ((*xinfo)[2 * (xk - 1)] & 31u) == 0 && xlog < 32)
      slot = tc_xslot(op, uint16_t(d));
    uint32_t a_eff = a;
    if (op == OP_V_EXTRACT32 || op == OP_V_EXTRACT64) {   // a lane of a v128 = a cell move
      a_eff = a + (op == OP_V_EXTRACT32 ? d : 2 * d);
      slot = tc_slot(op == OP_V_EXTRACT32 ? OP_MOV32 : OP_MOV64);
    }
    if (!slot) continue;
    TInstr &t = tc[pc];
    uint32_t *w = t.w;
    w[1] = off(a_eff); w[2] = off(b); w[3] = off(c); w[4] = imm; w[5] = 0; w[6] = cnt; w[7] = 0;
    if (op == OP_I32_ADD3 || op == OP_SELECT32 || op == OP_SELECT64 ||
        op == OP_I32_ADD_XROTR_I || op == OP_I32_ADD3_XROTR_I)
      w[5] = off(d);
    if (op == OP_I32_ADD3_XROTR_I) {   // the 4th operand (y) is read by the handler itself
      w[7] = off(imm & 0xFFFFu);
      w[4] = imm >> 16;
    }
    if (is_branch(op)) {
      const int32_t taken = int32_t(cnt) + int32_t(int16_t(d));
      if (taken < 0 || imm >= (1u << 26)) continue;
      w[4] = imm * 32u;
      w[7] = uint32_t(taken);
      if (op >= OP_BR_EQ_I && op <= OP_BR_GE_U_I) {
        w[3] = uint32_t(int32_t(int16_t(b)));
        w[2] = 0;
      } else {
        w[3] = 0;
      }
    } else if (const uint32_t n = mem_bytes(op)) {
      const uint64_t last = uint64_t(imm) + n - 1;
      if (last > 0xFFFFFFFFull) continue;
      w[7] = uint32_t(last);
    } else if (op == OP_XLD || op == OP_XST) {   // (xop: a slot was found above)
      const uint64_t last = uint64_t(imm) + mem_bytes(uint16_t(d)) - 1;
      if (last > 0xFFFFFFFFull) continue;
      w[7] = uint32_t(last);
      w[5] = (*xinfo)[2 * (xk - 1)] | xlog;       // word offset | granule log
      w[op == OP_XLD ? 2 : 3] = P.xmems[xk - 1].min;   // (the other field: the value / result cell)
    } else if (op == OP_CONST64) {
      w[7] = I.w1;   // high word
      w[1] = w[2] = 0;
    } else if (op == OP_CONST32) {
      w[1] = w[2] = 0;
    } else if (op == OP_V_REPLACE64) {
      w[7] = d;      // the lane
      if (d > 1) continue;
    } else if (op == OP_I32_ROTL_I || op == OP_I32_XOR_ROTL_I) {
      w[4] = (32u - (imm & 31u)) & 31u;     // rotl k == rotr -k
    }
    if (op == OP_CALL || op == OP_RET || op == OP_POST_CALL) {   // gen_tc.py call handlers
      const uint32_t fb = P.global_cells;
      if (a >= T || fb >= T) continue;
      w[1] = a * unit;
      w[2] = fb * unit;
      w[3] = b;                                   // RET / POST_CALL: result cells
      w[4] = 0; w[5] = 0; w[7] = 0;
      if (op == OP_CALL) {
        if (imm >= (1u << 26) || a < fb) continue;
        w[3] = ((uint32_t(pc) + 1) & 0xFFFFFu) | (a << 20);   // return record
        w[4] = imm * 32u;
        w[7] = b | (c << 16);                     // nargs | nlocals << 16
      }
    }
    if (op == OP_TAIL_CALL) {   // gen_tc.py tail_call_body (WB_TC_TAIL=0: the C++ step, A/B aid)
      const uint32_t fb = P.global_cells;
      if (tail_off || a >= T || fb >= T || a < fb || imm >= (1u << 26) || b > 0xFFFFu) continue;
      w[1] = a * unit;
      w[2] = fb * unit;
      w[3] = 0; w[5] = 0;
      w[4] = imm * 32u;
      w[7] = b | (c << 16);                       // nargs | locals to zero << 16
    }
    w[0] = uint32_t(slot) * TC_SLOT_BYTES;
    code[pc].w0 |= DBC_HOT;
  }
  // Pipelined ARX pairs: ADD_XROTR falling into ADD3_XROTR prefetches the latter's 4th
  // operand. The *_E handler relies on that, so it must only ever be entered by that
  // fall-through: not a jump/call/return target, and not an entry point of the core
  // (DBC_HOT cleared: a run that stops in front of it resumes in the C++ step).
  const size_t n = P.code.size();
  const std::vector<uint8_t> target = jump_targets(P);
  // V blob: fused pair handlers (gen_tc.py PAIRS) for an instruction and the one after
  // it; the instruction at pc + 1 keeps its own handler for jumps and resumes
  if (vframe) {
    std::vector<int> sl(n);
    for (size_t pc = 0; pc < n; pc++) sl[pc] = int(tc[pc].w[0] / TC_SLOT_BYTES);
    for (size_t pc = 0; pc < n; pc++) {
      size_t m = 0;   // handled instructions from pc on (a tuple only covers those)
      // a tuple never covers the start of a compiled run (jit.cpp replaces that TInstr)
      while (pc + m < n && m < 8 && sl[pc + m] && !(m && run_start && (*run_start)[pc + m])) m++;
      int len = 0;
      const int ps = m >= 2 ? tc_tuple_slot(&sl[pc], int(m), &len) : 0;
      if (ps) tc[pc].w[0] = uint32_t(ps) * TC_SLOT_BYTES;
    }
  }
  for (size_t pc = 1; pc < n && !vframe; pc++) {
    const uint16_t op = uint16_t(P.code[pc].w0 & 0x7FFFu), prev = uint16_t(P.code[pc - 1].w0 & 0x7FFFu);
    if (op == OP_I32_ADD3_XROTR_I && prev == OP_I32_ADD_XROTR_I && !target[pc] &&
        tc[pc].w[0] && tc[pc - 1].w[0]) {
      tc[pc - 1].w[0] = TC_SLOT_I32_ADD_XROTR_I_PF4 * TC_SLOT_BYTES;
      tc[pc].w[0] = TC_SLOT_I32_ADD3_XROTR_I_E * TC_SLOT_BYTES;
      code[pc].w0 &= ~DBC_HOT;
    }
  }
  return tc;
}

}  // namespace wb
