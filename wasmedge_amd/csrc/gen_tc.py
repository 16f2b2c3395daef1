#!/usr/bin/env python3
"""Generator of the direct-threaded gfx950 dispatch core (tc = "threaded code").

Why: on CDNA4 a wave issues one instruction per ~4 cycles and every scalar branch costs
15-30 cycles (tools/ubench/lat.hip). The compiled C++ dispatch loop walks a binary
compare tree over ~330 opcodes (≈9 compare+branch pairs) and waits for each
instruction's LDS operands serially: ≈526 cycles per dispatch on C2 (profiles/r01b_*).
This core replaces that, for the hot opcodes, with hand-written handlers:

  * direct threading: every 32-byte threaded instruction (TInstr, see tc.h) carries its
    handler's byte offset; dispatch is `s_add/s_addc/s_setpc_b64` (no compare tree);
  * fixed 256-byte handler slots, laid out in four banks: {converged, diverged} x
    {A, B}. The instruction being executed sits in SGPR bank A or B; its handler
    prefetches the fall-through successor into the other bank, so no SGPR copies;
  * software-pipelined operands: a handler issues the LDS reads of the NEXT
    instruction's operands (a, b, d; each a ds_read2_b32 of cells k and k+1) before it
    dispatches, so their latency overlaps the dispatch itself;
  * the "diverged" banks additionally stop when the uniform pc reaches the lowest pc of
    the waiting lanes (min-pc reconvergence, see batch_kernel.hip).

Anything a handler cannot finish for every active lane (an opcode without a handler, a
branch whose lanes disagree, a misaligned or out-of-bounds access) leaves the core
BEFORE the instruction has any effect; the compiled C++ step (dbc_step.inc) then
executes it with full per-lane semantics. So the core never traps, and every result it
produces is one the C++ step would produce.

Outputs (both written next to this file; run by the Makefile):
  tc_blob.inc   the handler blob as a C string for a file-scope asm() (device pass only)
  tc_slots.h    opcode -> slot map for the host translator (tc.cpp)
"""
import os
import re
import sys

SLOT = 256                         # bytes per handler slot
JIT_XS = 64                        # offset of the xs exit stub in slot 0 (V blob)
HERE = os.path.dirname(os.path.abspath(__file__))

# ---------------------------------------------------------------- register conventions
# SGPRs (all clobbered by the kernel's asm statement)
CODE = "s[60:61]"     # TInstr array base
PCOFF = "s62"         # current pc * 32
OTHER = "s63"         # lowest waiting pc * 32 (diverged banks stop there)
LIM = "s64"           # count limit: leave at a taken branch once CNT >= LIM
CNT = "s65"           # wasm instructions retired in this call
RET = "s[66:67]"      # return address into the kernel
T = ("s68", "s69")    # temp pair (dispatch target)
TP = "s[68:69]"
BA = ("s70", "s71")   # bank-A handler base of the current mode
BB = ("s72", "s73")   # bank-B handler base
T2 = "s[74:75]"       # temp pair (lane masks)
T2L, T2H = "s74", "s75"
IA = 76               # s[76:83] instruction in bank A (w0..w7)
IB = 84               # s[84:91] instruction in bank B
REASON = "s92"        # 0: execute pc in the C++ step; 1: back to the scheduler
# VGPRs (v104..v127, clobbered)
FR = "v104"           # LDS byte address of this lane's cell 0
PAGES = "v105"        # this lane's memory size in pages
MEM = "v[106:107]"    # this lane's linear-memory word 0 (lane-interleaved)
A = ("v108", "v109"); AP = "v[108:109]"   # operand a: cells a, a+1
B = ("v110", "v111"); BP = "v[110:111]"   # operand b
D = ("v112", "v113"); DP = "v[112:113]"   # operand d
R = ("v114", "v115"); RP = "v[114:115]"   # result
W = ("v116", "v117"); WP = "v[116:117]"   # word index, 0 (v117 is always 0)
X = ("v118", "v119"); XP = "v[118:119]"   # temps / 64-bit address
Y = ("v120", "v121"); YP = "v[120:121]"
AADDR, BADDR, DADDR, CADDR = "v122", "v123", "v124", "v125"
Z = ("v126", "v127"); ZP = "v[126:127]"
GSP = "v102"          # this lane's call-stack depth (slots), in/out
MSH1 = "v99"          # linear-memory granule: 2 + g (the wave interleaves its lanes'
MSH2 = "v100"         # memories in granules of 4 << g bytes); 8 + g (bytes per granule row)
HWM = "v101"          # one past the highest memory byte written (LS_HWM), in/out
SB0 = "v103"          # LDS byte address of this lane's call-stack slot 0
SLDS = "s93"          # call-stack slots held in LDS (the fast path stays below this)
VSYNC = "s94"         # V frames: (VMAX - frame cells) * 8, the frame-sync jump offset
LOW = "s95"           # lowest waiting pc * 32 (<= OTHER; a jump to or below it re-aims OTHER)
# V frames only: the lanes in the core (ALL, their frames are in v128..) and, at entry and
# exit, the group that runs (GROUP, = the T2 temp pair); VPC / VCNT: per-lane pc of the
# lanes waiting in the core and per-lane wasm-instruction count not yet in CNT (SIMT mode,
# jit.cpp Lsched; both are outputs of every core call)
ALL = "s[96:97]"
GROUP = T2
VPC = "v92"
VCNT = "v93"


def sreg(bank, k):
    return "s%d" % ((IA if bank == "A" else IB) + k)


def sbank(bank):
    b = IA if bank == "A" else IB
    return "s[%d:%d]" % (b, b + 7)


# ---------------------------------------------------------------- handler specs
# Each spec: name -> (DBC op names it serves, body function(g) -> list of lines).
# A body runs after `s_waitcnt lgkmcnt(0)` (operands of this instruction are in A/B/D,
# the prefetched successor is in the other bank). It ends with one of the tails:
#   g.next()        fall through (count cnt, pc += 1)
#   g.exit_here()   leave before this instruction had any effect
#   explicit branch code using g.taken(...)


VB = 128               # V-frame blob: frame cell i of the lane lives in VGPR v[VB + i]
VMAX = 128             # cells a V frame can hold (v128..v255)
SELF = "#self-fetch"   # first line of a V body that fetches its own operands


class Gen:
    def __init__(self, mode, bank, vf=False):
        self.mode, self.bank = mode, bank          # mode "C" converged / "D" diverged
        self.other = "B" if bank == "A" else "A"
        self.n = 0
        self.vf = vf                               # frame in VGPRs (GPR-index mode)
        self.pre = "Lvf" if vf else "Ltc"
        self.stubs = bank                          # whose exit stubs (slot 0) it uses
        self.glue = False                          # first half of a fused pair

    def x(self, k):                                # field k of the current instruction
        return sreg(self.bank, k)

    def y(self, k):                                # field k of the successor bank
        return sreg(self.other, k)

    _uid = [0]

    def lab(self, tag):
        Gen._uid[0] += 1
        return "%s_%s_%d" % (self.pre, tag, Gen._uid[0])

    def exit_here(self):
        return ["s_branch %s" % self.xh()]

    def xh(self):     # exit stubs live in slot 0 of every bank (s_branch reaches +-128 KB)
        return "%s_xh_%s%s" % (self.pre, self.mode, self.stubs)

    def xs(self):
        return "%s_xs_%s%s" % (self.pre, self.mode, self.stubs)

    # -- V frames: cells are VGPRs v[VB + cell], addressed through GPR-index mode with
    # the cell index in an SGPR (instruction fields hold cell indices, not LDS offsets).
    # While index mode is on, EVERY VALU operand it names is offset, so each sequence
    # holds nothing but the indexed moves and is closed before any other VALU or branch.
    def vread(self, sidx, regs, base=VB):
        """regs[k] = v[base + k + idx]; sidx: SGPR holding the cell index."""
        return ["s_set_gpr_idx_on %s, gpr_idx(SRC0)" % sidx] + \
            ["v_mov_b32 %s, v%d" % (r, base + k) for k, r in enumerate(regs)] + ["s_set_gpr_idx_off"]

    def vwrites(self, items):
        """items: [(SGPR cell index, [value regs])]: v[VB + idx + k] = regs[k]."""
        out = []
        for i, (sidx, regs) in enumerate(items):
            out.append("s_set_gpr_idx_on %s, gpr_idx(DST)" % sidx if i == 0 else
                       "s_set_gpr_idx_idx %s" % sidx)
            out += ["v_mov_b32 v%d, %s" % (VB + k, r) for k, r in enumerate(regs)]
        return out + ["s_set_gpr_idx_off"]

    def vprologue(self, body):
        """Fetch the operands (a: field 1, b: field 2, d: field 5; cells k, k+1) that
        `body` names -- in the LDS blob the previous handler prefetched all of them."""
        out, on = [], False
        text = "\n".join(body)
        for field, regs, pair in ((1, A, AP), (2, B, BP), (5, D, DP)):
            # a register by name, or the pair "v[lo:hi]" (64-bit operands) for both
            both = pair in text
            need = [both or re.search(r"\b%s\b" % r, text) is not None for r in regs]
            if not any(need):
                continue
            out.append("s_set_gpr_idx_idx %s" % self.x(field) if on else
                       "s_set_gpr_idx_on %s, gpr_idx(SRC0)" % self.x(field))
            on = True
            out += ["v_mov_b32 %s, v%d" % (r, VB + k) for k, r in enumerate(regs) if need[k]]
        return out + (["s_set_gpr_idx_off"] if on else [])

    def issue_reads(self, bank):
        """LDS reads of the operands of the instruction in `bank` (fields 1, 2, 5)."""
        f = lambda k: sreg(bank, k)
        return ["v_add_u32 %s, %s, %s" % (AADDR, f(1), FR),
                "v_add_u32 %s, %s, %s" % (BADDR, f(2), FR),
                "v_add_u32 %s, %s, %s" % (DADDR, f(5), FR),
                "ds_read2_b32 %s, %s offset1:64" % (AP, AADDR),
                "ds_read2_b32 %s, %s offset1:64" % (BP, BADDR),
                "ds_read2_b32 %s, %s offset1:64" % (DP, DADDR)]

    def dispatch(self, bank):
        base = BA if bank == "A" else BB
        return ["s_add_u32 %s, %s, %s" % (T[0], base[0], sreg(bank, 0)),
                "s_addc_u32 %s, %s, 0" % (T[1], base[1]),
                "s_setpc_b64 %s" % TP]

    def next(self, cnt=True, pf4=False):
        if self.glue:
            # first half of a fused pair (V blob, converged mode): retire it, make the
            # second the current instruction (other bank, loaded by the predecessor)
            # and start loading the one after into this bank
            return ["s_add_u32 %s, %s, %s" % (CNT, CNT, self.x(6)),
                    "s_add_u32 %s, %s, 32" % (PCOFF, PCOFF), "s_waitcnt lgkmcnt(0)",
                    "s_load_dwordx8 %s, %s, %s offset:0x20" % (sbank(self.bank), CODE, PCOFF)]
        """Fall through to the prefetched successor (other bank). pf4: also read the
        successor's 4th operand (field 7) into Y0, its address kept in X1 (only for
        successors the translator gave an *_E handler, see tc.cpp)."""
        out = []
        if cnt:
            out.append("s_add_u32 %s, %s, %s" % (CNT, CNT, self.x(6)))
        out.append("s_add_u32 %s, %s, 32" % (PCOFF, PCOFF))
        if self.mode == "D":
            out += ["s_cmp_ge_u32 %s, %s" % (PCOFF, OTHER), "s_cbranch_scc1 %s" % self.xs()]
        if self.vf:
            # the successor's fields (loaded two dispatches ago) must be resident; no
            # operand prefetch: the successor reads its operands from VGPRs itself
            out.append("s_waitcnt lgkmcnt(0)")
        else:
            out += self.issue_reads(self.other)
        if pf4 and not self.vf:
            out += ["v_add_u32 %s, %s, %s" % (X[1], sreg(self.other, 7), FR),
                    "ds_read_b32 %s, %s" % (Y[0], X[1])]
        # prefetch the successor's successor into this bank (its fields are dead now)
        out.append("s_load_dwordx8 %s, %s, %s offset:0x20" % (sbank(self.bank), CODE, PCOFF))
        out += self.dispatch(self.other)
        return out

    def taken(self, target, cnt):
        """Uniform jump to byte offset `target` (SGPR), adding count `cnt` (SGPR)."""
        out = ["s_mov_b32 %s, %s" % (PCOFF, target),
               "s_add_u32 %s, %s, %s" % (CNT, CNT, cnt),
               "s_cmp_ge_u32 %s, %s" % (CNT, LIM), "s_cbranch_scc1 %s" % self.xs()]
        if self.mode == "D":
            # a jump back to or below every waiting lane next meets the lowest of them
            out += ["s_cmp_le_u32 %s, %s" % (PCOFF, LOW),
                    "s_cselect_b32 %s, %s, %s" % (OTHER, LOW, OTHER),
                    "s_cmp_ge_u32 %s, %s" % (PCOFF, OTHER), "s_cbranch_scc1 %s" % self.xs()]
        # the successor prefetch into the other bank must have landed before both banks
        # are reloaded (SMEM returns out of order: a late stale load would win). The LDS
        # blob waited at handler entry; the V-frame blob waits here.
        if self.vf:
            out.append("s_waitcnt lgkmcnt(0)")
        out += ["s_load_dwordx8 %s, %s, %s" % (sbank(self.other), CODE, PCOFF),
                "s_load_dwordx8 %s, %s, %s offset:0x20" % (sbank(self.bank), CODE, PCOFF),
                "s_waitcnt lgkmcnt(0)"]
        if not self.vf:
            out += self.issue_reads(self.other)
        out += self.dispatch(self.other)
        return out

    # -- result writes
    def w32(self, v=None):
        if self.vf:
            return self.vwrites([(self.x(3), [v or R[0]])])
        return ["v_add_u32 %s, %s, %s" % (CADDR, self.x(3), FR),
                "ds_write_b32 %s, %s" % (CADDR, v or R[0])]

    def w64(self, lo=None, hi=None):
        if self.vf:
            return self.vwrites([(self.x(3), [lo or R[0], hi or R[1]])])
        return ["v_add_u32 %s, %s, %s" % (CADDR, self.x(3), FR),
                "ds_write2_b32 %s, %s, %s offset1:64" % (CADDR, lo or R[0], hi or R[1])]

    def w128(self, lo, hi):
        """lo/hi: VGPR pair names (cells c, c+1 and c+2, c+3)."""
        if self.vf:
            return self.vwrites([(self.x(3), [lo[0], lo[1], hi[0], hi[1]])])
        return ["v_add_u32 %s, %s, %s" % (CADDR, self.x(3), FR),
                "ds_write2_b32 %s, %s, %s offset1:64" % (CADDR, lo[0], lo[1]),
                "ds_write2_b32 %s, %s, %s offset0:128 offset1:192" % (CADDR, hi[0], hi[1])]

    def bool_result(self):
        return ["v_cndmask_b32_e64 %s, 0, 1, vcc" % R[0]] + self.w32()

    def cond_branch(self, cmp_lines):
        """cmp_lines set vcc per lane (true = taken). Uniform outcome -> branch or fall
        through; lanes that disagree -> leave (the C++ step splits the wave)."""
        nt = self.lab("nt")
        return cmp_lines + [
            "s_and_b64 %s, vcc, exec" % T2,            # SCC = any lane takes it
            "s_cbranch_scc0 %s" % nt,
            "s_cmp_eq_u64 %s, exec" % T2,
            "s_cbranch_scc0 %s" % self.xh(),             # split decision
        ] + self.taken(self.x(4), self.x(7)) + ["%s:" % nt] + self.next()


I32_BIN = {  # name -> (instruction template over (d, a, b)), b may be an SGPR
    "ADD": "v_add_u32_e64 {d}, {a}, {b}",
    "SUB": "v_sub_u32_e64 {d}, {a}, {b}",
    "MUL": "v_mul_lo_u32 {d}, {a}, {b}",
    "AND": "v_and_b32_e64 {d}, {a}, {b}",
    "OR": "v_or_b32_e64 {d}, {a}, {b}",
    "XOR": "v_xor_b32_e64 {d}, {a}, {b}",
    "SHL": "v_lshlrev_b32_e64 {d}, {b}, {a}",
    "SHR_S": "v_ashrrev_i32_e64 {d}, {b}, {a}",
    "SHR_U": "v_lshrrev_b32_e64 {d}, {b}, {a}",
    "ROTR": "v_alignbit_b32 {d}, {a}, {a}, {b}",
}
CMP = {"EQ": "eq_u", "NE": "ne_u", "LT_S": "lt_i", "LT_U": "lt_u", "GT_S": "gt_i",
       "GT_U": "gt_u", "LE_S": "le_i", "LE_U": "le_u", "GE_S": "ge_i", "GE_U": "ge_u"}


def specs():
    S = []   # (slot name, [dbc ops], body)

    def add(name, ops, body, slots=1):
        S.append((name, ops, body))
        for k in range(1, slots):            # a handler may span several slots
            S.append((name + "+%d" % k, [], None))

    # ---- control
    add("NOP_CNT", ["NOP_CNT"], lambda g: g.next())
    add("JMP", ["JMP"], lambda g: g.taken(g.x(4), g.x(7)))
    add("BR_IF", ["BR_IF"], lambda g: g.cond_branch(["v_cmp_ne_u32_e64 vcc, 0, %s" % A[0]]))
    add("BR_UNLESS", ["BR_UNLESS"],
        lambda g: g.cond_branch(["v_cmp_eq_u32_e64 vcc, 0, %s" % A[0]]))
    for c, k in CMP.items():
        add("BR_" + c, ["BR_" + c],
            lambda g, k=k: g.cond_branch(["v_cmp_%s32_e64 vcc, %s, %s" % (k, A[0], B[0])]))
        add("BR_%s_I" % c, ["BR_%s_I" % c],
            lambda g, k=k: g.cond_branch(["v_cmp_%s32_e64 vcc, %s, %s" % (k, A[0], g.x(3))]))
    # ---- moves / constants / select
    add("MOV32", ["MOV32"], lambda g: g.w32(A[0]) + g.next())
    add("MOV64", ["MOV64"], lambda g: g.w64(A[0], A[1]) + g.next())
    add("CONST32", ["CONST32"], lambda g: ["v_mov_b32 %s, %s" % (R[0], g.x(4))] + g.w32() + g.next())
    add("CONST64", ["CONST64"], lambda g: ["v_mov_b32 %s, %s" % (R[0], g.x(4)),
                                           "v_mov_b32 %s, %s" % (R[1], g.x(7))] + g.w64() + g.next())
    add("SELECT32", ["SELECT32"], lambda g: [
        "v_cmp_ne_u32_e64 vcc, 0, %s" % D[0],
        "v_cndmask_b32_e64 %s, %s, %s, vcc" % (R[0], B[0], A[0])] + g.w32() + g.next())
    add("SELECT64", ["SELECT64"], lambda g: [
        "v_cmp_ne_u32_e64 vcc, 0, %s" % D[0],
        "v_cndmask_b32_e64 %s, %s, %s, vcc" % (R[0], B[0], A[0]),
        "v_cndmask_b32_e64 %s, %s, %s, vcc" % (R[1], B[1], A[1])] + g.w64() + g.next())
    # ---- i32
    for nm, t in I32_BIN.items():
        add("I32_" + nm, ["I32_" + nm],
            lambda g, t=t: [t.format(d=R[0], a=A[0], b=B[0])] + g.w32() + g.next())
        add("I32_%s_I" % nm, ["I32_%s_I" % nm],
            lambda g, t=t: [t.format(d=R[0], a=A[0], b=g.x(4))] + g.w32() + g.next())
    add("I32_ROTL", ["I32_ROTL"], lambda g: [
        "v_sub_u32_e64 %s, 0, %s" % (X[0], B[0]),
        "v_alignbit_b32 %s, %s, %s, %s" % (R[0], A[0], A[0], X[0])] + g.w32() + g.next())
    for c, k in CMP.items():
        add("I32_" + c, ["I32_" + c], lambda g, k=k: [
            "v_cmp_%s32_e64 vcc, %s, %s" % (k, A[0], B[0])] + g.bool_result() + g.next())
        add("I32_%s_I" % c, ["I32_%s_I" % c], lambda g, k=k: [
            "v_cmp_%s32_e64 vcc, %s, %s" % (k, A[0], g.x(4))] + g.bool_result() + g.next())
    add("I32_EQZ", ["I32_EQZ"], lambda g: ["v_cmp_eq_u32_e64 vcc, 0, %s" % A[0]] +
        g.bool_result() + g.next())
    add("I32_ADD3", ["I32_ADD3"], lambda g: [
        "v_add3_u32 %s, %s, %s, %s" % (R[0], A[0], B[0], D[0])] + g.w32() + g.next())
    add("I32_XOR_ROTR_I", ["I32_XOR_ROTR_I"], lambda g: [
        "v_xor_b32_e32 %s, %s, %s" % (X[0], A[0], B[0]),
        "v_alignbit_b32 %s, %s, %s, %s" % (R[0], X[0], X[0], g.x(4))] + g.w32() + g.next())
    # ARX pairs: sum -> c, then d (or the 4th cell y, read here) = rotr(. ^ sum, k)
    def add_xrotr(g, pf4=False):
        out = ["v_add_u32_e32 %s, %s, %s" % (R[0], A[0], B[0]),
               "v_xor_b32_e32 %s, %s, %s" % (X[0], D[0], R[0]),
               "v_alignbit_b32 %s, %s, %s, %s" % (R[1], X[0], X[0], g.x(4))]
        if g.vf:   # operands b, d read as indexed sources; d's new value written indexed
            return [SELF, "s_set_gpr_idx_on %s, gpr_idx(SRC0)" % g.x(1), "v_mov_b32 %s, v%d" % (A[0], VB),
                    "s_set_gpr_idx_idx %s" % g.x(2), "v_add_u32_e32 %s, v%d, %s" % (R[0], VB, A[0]),
                    "s_set_gpr_idx_idx %s" % g.x(5), "v_xor_b32_e32 %s, v%d, %s" % (X[0], VB, R[0]),
                    "s_set_gpr_idx_on %s, gpr_idx(DST)" % g.x(3), "v_mov_b32 v%d, %s" % (VB, R[0]),
                    "s_set_gpr_idx_idx %s" % g.x(5),
                    "v_alignbit_b32 v%d, %s, %s, %s" % (VB, X[0], X[0], g.x(4)),
                    "s_set_gpr_idx_off"] + g.next()
        return out + g.w32() + ["v_add_u32 %s, %s, %s" % (DADDR, g.x(5), FR),
                                "ds_write_b32 %s, %s" % (DADDR, R[1])] + g.next(pf4=pf4)

    def add3_xrotr(g, pre=True):
        """pre: read the 4th cell y here (else the PF4 predecessor read it into Y0)."""
        if g.vf:
            return [SELF, "s_set_gpr_idx_on %s, gpr_idx(SRC0)" % g.x(1), "v_mov_b32 %s, v%d" % (A[0], VB),
                    "s_set_gpr_idx_idx %s" % g.x(2), "v_mov_b32 %s, v%d" % (B[0], VB),
                    "s_set_gpr_idx_idx %s" % g.x(5),
                    "v_add3_u32 %s, v%d, %s, %s" % (R[0], VB, A[0], B[0]),
                    "s_set_gpr_idx_idx %s" % g.x(7), "v_xor_b32_e32 %s, v%d, %s" % (X[0], VB, R[0]),
                    "s_set_gpr_idx_on %s, gpr_idx(DST)" % g.x(3), "v_mov_b32 v%d, %s" % (VB, R[0]),
                    "s_set_gpr_idx_idx %s" % g.x(7),
                    "v_alignbit_b32 v%d, %s, %s, %s" % (VB, X[0], X[0], g.x(4)),
                    "s_set_gpr_idx_off"] + g.next()
        out = ["v_add_u32 %s, %s, %s" % (X[1], g.x(7), FR), "ds_read_b32 %s, %s" % (Y[0], X[1])] \
            if pre else []
        out += ["v_add3_u32 %s, %s, %s, %s" % (R[0], A[0], B[0], D[0])] + g.w32()
        if pre:
            out.append("s_waitcnt lgkmcnt(0)")
        return out + ["v_xor_b32_e32 %s, %s, %s" % (X[0], Y[0], R[0]),
                      "v_alignbit_b32 %s, %s, %s, %s" % (R[1], X[0], X[0], g.x(4)),
                      "ds_write_b32 %s, %s" % (X[1], R[1])] + g.next()

    add("I32_ADD_XROTR_I", ["I32_ADD_XROTR_I"], add_xrotr)
    add("I32_ADD3_XROTR_I", ["I32_ADD3_XROTR_I"], add3_xrotr)
    # pipelined pair (tc.cpp picks these when ADD_XROTR falls into ADD3_XROTR and the
    # latter is no jump target): the first prefetches the second's 4th operand y.
    # (LDS blob only; the V-frame translation never selects them.)
    add("I32_ADD_XROTR_I_PF4", [], lambda g: add_xrotr(g, pf4=True))
    add("I32_ADD3_XROTR_I_E", [], lambda g: add3_xrotr(g, pre=False))
    # ---- calls (dbc_step.inc OP_CALL / OP_RET / OP_POST_CALL, LDS part of the call stack
    # only; anything else -- HBM slots, divergent return targets, leaving the entry
    # function -- leaves the core before any effect). Fields (tc.cpp): w1 = L or the
    # result cell, w2 = frame base fb (cell offsets); CALL: w3 = return record,
    # w4 = target*32, w7 = nargs | nlocals << 16; RET/POST_CALL: w3 = result cells.
    def copy(src, dst, cnt, tag, g, step="0x100", sub=False):
        top, end = g.lab(tag), g.lab(tag + "e")
        mv = "v_subrev_u32_e32" if sub else "v_add_u32_e32"
        return ["%s:" % top, "s_cmp_eq_u32 %s, 0" % cnt, "s_cbranch_scc1 %s" % end,
                "ds_read_b32 %s, %s" % (Y[0], src), "s_waitcnt lgkmcnt(0)",
                "ds_write_b32 %s, %s" % (dst, Y[0]),
                "%s %s, %s, %s" % (mv, src, step, src), "%s %s, %s, %s" % (mv, dst, step, dst),
                "s_sub_u32 %s, %s, 1" % (cnt, cnt), "s_branch %s" % top, "%s:" % end]

    def lds_guard(g, vreg):     # leave unless every active lane's vreg <= SLDS
        return ["v_cmp_lt_u32_e64 vcc, %s, %s" % (SLDS, vreg),
                "s_and_b64 %s, vcc, exec" % T2, "s_cbranch_scc1 %s" % g.xh()]

    # V frames: the same protocol, frame cells moved with GPR-index moves. Fields hold
    # cell indices: w1 = L (RET: the result cell), w2 = fb.
    def vloop(g, tag, cnt, body):
        """while (cnt--) body -- cnt: SGPR, body: lines (no VALU left in index mode)."""
        top, end = g.lab(tag), g.lab(tag + "e")
        return ["%s:" % top, "s_cmp_eq_u32 %s, 0" % cnt, "s_cbranch_scc1 %s" % end] + body + \
            ["s_sub_u32 %s, %s, 1" % (cnt, cnt), "s_branch %s" % top, "%s:" % end]

    def vmove(g, tag, cnt, si, di, step):
        """v[VB+di] = v[VB+si], cnt times, indices stepping by `step` (1 / -1)."""
        op = "s_add_u32" if step > 0 else "s_sub_u32"
        return vloop(g, tag, cnt, g.vread(si, [Y[0]]) + g.vwrites([(di, [Y[0]])]) +
                     ["%s %s, %s, 1" % (op, si, si), "%s %s, %s, 1" % (op, di, di)])

    def call_body_v(g):
        n, n1, si, di = "s68", "s69", T2L, T2H
        out = ["s_sub_u32 %s, %s, %s" % (n, g.x(1), g.x(2)),
               "s_add_u32 %s, %s, 1" % (n1, n),
               "v_add_u32_e64 %s, %s, %s" % (X[0], n1, GSP)] + lds_guard(g, X[0])
        out += ["v_lshl_add_u32 %s, %s, 8, %s" % (X[1], GSP, SB0),     # &stack[gsp]
                "s_mov_b32 %s, %s" % (si, g.x(2))]
        out += vloop(g, "sp", n, g.vread(si, [Y[0]]) + [               # spill [fb, L)
            "ds_write_b32 %s, %s" % (X[1], Y[0]), "v_add_u32_e32 %s, 0x100, %s" % (X[1], X[1]),
            "s_add_u32 %s, %s, 1" % (si, si)])
        out += ["v_mov_b32 %s, %s" % (Y[1], g.x(3)), "ds_write_b32 %s, %s" % (X[1], Y[1]),
                "v_add_u32_e64 %s, %s, %s" % (GSP, n1, GSP),
                "s_and_b32 %s, %s, 0xffff" % (n, g.x(7)),
                "s_mov_b32 %s, %s" % (si, g.x(1)), "s_mov_b32 %s, %s" % (di, g.x(2))]
        out += vmove(g, "ar", n, si, di, 1)                            # args -> fb
        out += ["s_lshr_b32 %s, %s, 16" % (n, g.x(7)), "v_mov_b32 %s, 0" % Y[0]]
        out += vloop(g, "zl", n, g.vwrites([(di, [Y[0]])]) + ["s_add_u32 %s, %s, 1" % (di, di)])
        return out + g.taken(g.x(4), g.x(6))

    def ret_record(g, t):
        return lds_guard(g, GSP) + [
            "v_lshl_add_u32 %s, %s, 8, %s" % (X[1], GSP, SB0),
            "v_subrev_u32_e32 %s, 0x100, %s" % (X[1], X[1]),           # &stack[gsp - 1]
            "ds_read_b32 %s, %s" % (Y[1], X[1]), "s_waitcnt lgkmcnt(0)",
            # the raw record (pc | L << 20) must agree across lanes; readfirstlane reads
            # the loaded VGPR directly (a VALU-written VGPR would need wait states first)
            "v_readfirstlane_b32 %s, %s" % (t, Y[1]),
            "s_nop 1",                                   # VALU-written SGPR -> VALU read
            "v_cmp_ne_u32_e64 %s, %s, %s" % (T2, t, Y[1]),
            "s_and_b64 %s, %s, exec" % (T2, T2), "s_cbranch_scc1 %s" % g.xh(),   # split returns
            "s_and_b32 %s, %s, 0xfffff" % (t, t),
            "s_cmp_eq_u32 %s, 0xfffff" % t, "s_cbranch_scc1 %s" % g.xh(),   # entry function
            "v_subrev_u32_e32 %s, 1, %s" % (GSP, GSP)]

    def ret_body_v(g):
        t, si, di = "s68", T2L, T2H
        out = ret_record(g, t) + ["s_mov_b32 s69, %s" % g.x(3), "s_mov_b32 %s, %s" % (si, g.x(1)),
                                  "s_mov_b32 %s, %s" % (di, g.x(2))]
        out += vmove(g, "rr", "s69", si, di, 1)                        # results -> fb
        return out + ["s_lshl_b32 %s, %s, 5" % (t, t)] + g.taken(t, g.x(6))

    def post_call_body_v(g):
        n, r, si, di = "s68", "s69", T2L, T2H
        out = lds_guard(g, GSP) + [
            "s_sub_u32 %s, %s, %s" % (n, g.x(1), g.x(2)),
            "s_mov_b32 %s, %s" % (r, g.x(3)),
            # results fb.. -> L.. copied from the last one down (L > fb)
            "s_add_u32 %s, %s, %s" % (si, g.x(2), r), "s_sub_u32 %s, %s, 1" % (si, si),
            "s_add_u32 %s, %s, %s" % (di, g.x(1), r), "s_sub_u32 %s, %s, 1" % (di, di)]
        out += vmove(g, "pr", r, si, di, -1)
        out += ["v_subrev_u32_e64 %s, %s, %s" % (GSP, n, GSP),
                "v_lshl_add_u32 %s, %s, 8, %s" % (X[0], GSP, SB0),
                "s_mov_b32 %s, %s" % (di, g.x(2))]
        out += vloop(g, "rs", n, ["ds_read_b32 %s, %s" % (Y[0], X[0]), "s_waitcnt lgkmcnt(0)"] +
                     g.vwrites([(di, [Y[0]])]) +
                     ["v_add_u32_e32 %s, 0x100, %s" % (X[0], X[0]), "s_add_u32 %s, %s, 1" % (di, di)])
        return out + g.next()

    # return_call (dbc_step.inc OP_TAIL_CALL): the callee takes over the frame -- arguments
    # L.. -> fb.. (L >= fb: ascending is safe), its locals zeroed, no spill and no return
    # record. Fields: w1 = L, w2 = fb, w4 = target*32, w7 = nargs | nlocals << 16.
    def tail_call_body(g):
        n = "s68"
        if g.vf:
            si, di = T2L, T2H
            out = ["s_and_b32 %s, %s, 0xffff" % (n, g.x(7)),
                   "s_mov_b32 %s, %s" % (si, g.x(1)), "s_mov_b32 %s, %s" % (di, g.x(2))]
            out += vmove(g, "ar", n, si, di, 1)
            out += ["s_lshr_b32 %s, %s, 16" % (n, g.x(7)), "v_mov_b32 %s, 0" % Y[0]]
            out += vloop(g, "zl", n, g.vwrites([(di, [Y[0]])]) + ["s_add_u32 %s, %s, 1" % (di, di)])
            return out + g.taken(g.x(4), g.x(6))
        out = ["s_and_b32 %s, %s, 0xffff" % (n, g.x(7)),
               "v_add_u32_e64 %s, %s, %s" % (X[0], g.x(1), FR),
               "v_add_u32_e64 %s, %s, %s" % (X[1], g.x(2), FR)]
        out += copy(X[0], X[1], n, "ar", g)
        out += ["s_lshr_b32 %s, %s, 16" % (n, g.x(7)), "v_mov_b32 %s, 0" % Y[0]]
        zt, ze = g.lab("zl"), g.lab("zle")
        out += ["%s:" % zt, "s_cmp_eq_u32 %s, 0" % n, "s_cbranch_scc1 %s" % ze,
                "ds_write_b32 %s, %s" % (X[1], Y[0]), "v_add_u32_e32 %s, 0x100, %s" % (X[1], X[1]),
                "s_sub_u32 %s, %s, 1" % (n, n), "s_branch %s" % zt, "%s:" % ze]
        return out + g.taken(g.x(4), g.x(6))

    def call_body(g):
        if g.vf:
            return call_body_v(g)
        n, n1 = "s68", "s69"
        out = ["s_sub_u32 %s, %s, %s" % (n, g.x(1), g.x(2)), "s_lshr_b32 %s, %s, 8" % (n, n),
               "s_add_u32 %s, %s, 1" % (n1, n),
               "v_add_u32_e64 %s, %s, %s" % (X[0], n1, GSP)] + lds_guard(g, X[0])
        out += ["v_lshl_add_u32 %s, %s, 8, %s" % (X[1], GSP, SB0),     # &stack[gsp]
                "v_add_u32_e64 %s, %s, %s" % (X[0], g.x(2), FR)]       # &frame[fb]
        out += copy(X[0], X[1], n, "sp", g)                            # spill [fb, L)
        out += ["v_mov_b32 %s, %s" % (Y[1], g.x(3)), "ds_write_b32 %s, %s" % (X[1], Y[1]),
                "v_add_u32_e64 %s, %s, %s" % (GSP, n1, GSP),
                "s_and_b32 %s, %s, 0xffff" % (n, g.x(7)),
                "v_add_u32_e64 %s, %s, %s" % (X[0], g.x(1), FR),
                "v_add_u32_e64 %s, %s, %s" % (X[1], g.x(2), FR)]
        out += copy(X[0], X[1], n, "ar", g)                            # args -> fb
        out += ["s_lshr_b32 %s, %s, 16" % (n, g.x(7)), "v_mov_b32 %s, 0" % Y[0]]
        zt, ze = g.lab("zl"), g.lab("zle")
        out += ["%s:" % zt, "s_cmp_eq_u32 %s, 0" % n, "s_cbranch_scc1 %s" % ze,
                "ds_write_b32 %s, %s" % (X[1], Y[0]), "v_add_u32_e32 %s, 0x100, %s" % (X[1], X[1]),
                "s_sub_u32 %s, %s, 1" % (n, n), "s_branch %s" % zt, "%s:" % ze]
        return out + g.taken(g.x(4), g.x(6))

    def ret_body(g):
        if g.vf:
            return ret_body_v(g)
        t = "s68"
        out = lds_guard(g, GSP) + [
            "v_lshl_add_u32 %s, %s, 8, %s" % (X[1], GSP, SB0),
            "v_subrev_u32_e32 %s, 0x100, %s" % (X[1], X[1]),           # &stack[gsp - 1]
            "ds_read_b32 %s, %s" % (Y[1], X[1]), "s_waitcnt lgkmcnt(0)",
            # the raw record (pc | L << 20) must agree across lanes; readfirstlane reads
            # the loaded VGPR directly (a VALU-written VGPR would need wait states first)
            "v_readfirstlane_b32 %s, %s" % (t, Y[1]),
            "s_nop 1",                                   # VALU-written SGPR -> VALU read
            "v_cmp_ne_u32_e64 %s, %s, %s" % (T2, t, Y[1]),
            "s_and_b64 %s, %s, exec" % (T2, T2), "s_cbranch_scc1 %s" % g.xh(),   # split returns
            "s_and_b32 %s, %s, 0xfffff" % (t, t),
            "s_cmp_eq_u32 %s, 0xfffff" % t, "s_cbranch_scc1 %s" % g.xh(),   # entry function
            "v_subrev_u32_e32 %s, 1, %s" % (GSP, GSP),
            "s_mov_b32 s69, %s" % g.x(3),
            "v_add_u32_e64 %s, %s, %s" % (X[0], g.x(1), FR),
            "v_add_u32_e64 %s, %s, %s" % (X[1], g.x(2), FR)]
        out += copy(X[0], X[1], "s69", "rr", g)                       # results -> fb
        return out + ["s_lshl_b32 %s, %s, 5" % (t, t)] + g.taken(t, g.x(6))

    def post_call_body(g):
        if g.vf:
            return post_call_body_v(g)
        n, r = "s68", "s69"
        out = lds_guard(g, GSP) + [
            "s_sub_u32 %s, %s, %s" % (n, g.x(1), g.x(2)), "s_lshr_b32 %s, %s, 8" % (n, n),
            "s_mov_b32 %s, %s" % (r, g.x(3)),
            # results fb.. -> L.. copied from the last one down (L > fb)
            "s_lshl_b32 %s, %s, 8" % (T2L, r), "s_sub_u32 %s, %s, 0x100" % (T2L, T2L),
            "s_add_u32 %s, %s, %s" % (T2H, T2L, g.x(2)),
            "v_add_u32_e64 %s, %s, %s" % (X[0], T2H, FR),
            "s_add_u32 %s, %s, %s" % (T2H, T2L, g.x(1)),
            "v_add_u32_e64 %s, %s, %s" % (X[1], T2H, FR)]
        out += copy(X[0], X[1], r, "pr", g, sub=True)
        out += ["v_subrev_u32_e64 %s, %s, %s" % (GSP, n, GSP),
                "v_lshl_add_u32 %s, %s, 8, %s" % (X[0], GSP, SB0),
                "v_add_u32_e64 %s, %s, %s" % (X[1], g.x(2), FR)]
        out += copy(X[0], X[1], n, "rs", g)                            # restore [fb, L)
        return out + g.next()

    # ---- floating point. Results equal the reference's (x86 SSE as built by g++) except
    # for NaN payloads (DESIGN.md "Numerics"): a handler computes into registers, and if
    # any lane's result is a NaN it leaves before writing, so the compiled step produces
    # the exact payload; otherwise the IEEE result is the reference's.
    def nan_exit(g, pairs, w):
        """pairs: result registers (VGPR names or pairs) to test; w = 32 or 64."""
        out = []
        for k, r in enumerate(pairs):
            dst = T2 if k == 0 else "vcc"
            out.append("v_cmp_u_f%d_e64 %s, %s, %s" % (w, dst, r, r))
            if k:
                out.append("s_or_b64 %s, %s, vcc" % (T2, T2))
        return out + ["s_and_b64 %s, %s, exec" % (T2, T2), "s_cbranch_scc1 %s" % g.xh()]

    nan_labels = [0]

    def nan_fix(g, elems, w):
        """Exact NaN results in registers instead of leaving the core (the reference's
        x86 rule, dbc_ops.h nan_fix32/64): per element (r, a, b), a lane whose result is
        a NaN takes a quieted if a is a NaN, else b quieted if b is, else the default NaN
        with the sign set. Skipped with one compare + branch when no lane has a NaN.
        Clobbers the operand registers' high words and D (unused by binary ops)."""
        out = []
        hi = (lambda v: v) if w == 32 else (lambda v: "v" + v[2:-1].split(":")[1])
        lo = (lambda v: v) if w == 32 else (lambda v: "v" + v[2:-1].split(":")[0])
        q, dflt = ("0x400000", "0xffc00000") if w == 32 else ("0x80000", "0xfff80000")
        for r, a, b in elems:
            nan_labels[0] += 1
            lab = "Lnan_%d" % nan_labels[0]
            out += ["v_cmp_u_f%d_e64 %s, %s, %s" % (w, T2, r, r),
                    "s_and_b64 %s, %s, exec" % (T2, T2),
                    "s_cbranch_scc0 %s" % lab]
            if w == 64:
                out += ["v_mov_b32 %s, 0" % D[0]]
            out += ["v_mov_b32 %s, %s" % (D[1] if w == 64 else D[0], dflt)]
            for x in (b, a):   # a checked last: it wins
                out += ["v_cmp_u_f%d_e64 vcc, %s, %s" % (w, x, x),
                        "v_or_b32_e32 %s, %s, %s" % (hi(x), q, hi(x))]
                if w == 64:
                    out += ["v_cndmask_b32_e32 %s, %s, %s, vcc" % (D[0], D[0], lo(x)),
                            "v_cndmask_b32_e32 %s, %s, %s, vcc" % (D[1], D[1], hi(x))]
                else:
                    out += ["v_cndmask_b32_e32 %s, %s, %s, vcc" % (D[0], D[0], x)]
            if w == 64:
                out += ["v_cndmask_b32_e64 %s, %s, %s, %s" % (lo(r), lo(r), D[0], T2),
                        "v_cndmask_b32_e64 %s, %s, %s, %s" % (hi(r), hi(r), D[1], T2)]
            else:
                out += ["v_cndmask_b32_e64 %s, %s, %s, %s" % (r, r, D[0], T2)]
            out.append("%s:" % lab)
        return out

    def hi_reads(g, regs):
        """cells +2, +3 of the prefetched v128 operands (regs: [(addr, pair), ...])."""
        if g.vf:
            out = []
            for addr, pair in regs:
                lo, hi = pair[2:-1].split(":")
                out += g.vread(g.x(1 if addr == AADDR else 2), ["v" + lo, "v" + hi], base=VB + 2)
            return out
        return ["ds_read2_b32 %s, %s offset0:128 offset1:192" % (pair, addr) for addr, pair in regs] + \
            ["s_waitcnt lgkmcnt(0)"]

    FOPS = {"ADD": "v_add_f{w} {d}, {a}, {b}", "SUB": "v_add_f{w} {d}, {a}, -{b}",
            "MUL": "v_mul_f{w} {d}, {a}, {b}"}
    # add/sub/mul fix NaN results in place (nan_fix); the other FP ops still leave
    for nm, t in FOPS.items():
        add("F32_" + nm, ["F32_" + nm], lambda g, t=t: [
            t.format(w=32, d=R[0], a=A[0], b=B[0])] + nan_fix(g, [(R[0], A[0], B[0])], 32) +
            g.w32() + g.next(), slots=2)
        add("F64_" + nm, ["F64_" + nm], lambda g, t=t: [
            t.format(w=64, d=RP, a=AP, b=BP)] + nan_fix(g, [(RP, AP, BP)], 64) + g.w64() + g.next(),
            slots=2)
        add("V_F32X4_" + nm, ["V_F32X4_" + nm], lambda g, t=t: hi_reads(g, [(AADDR, XP), (BADDR, YP)]) + [
            t.format(w=32, d=R[0], a=A[0], b=B[0]), t.format(w=32, d=R[1], a=A[1], b=B[1]),
            t.format(w=32, d=Z[0], a=X[0], b=Y[0]), t.format(w=32, d=Z[1], a=X[1], b=Y[1])] +
            nan_fix(g, [(R[0], A[0], B[0]), (R[1], A[1], B[1]), (Z[0], X[0], Y[0]),
                        (Z[1], X[1], Y[1])], 32) + g.w128(R, Z) + g.next(), slots=3)
        add("V_F64X2_" + nm, ["V_F64X2_" + nm], lambda g, t=t: hi_reads(g, [(AADDR, XP), (BADDR, YP)]) + [
            t.format(w=64, d=RP, a=AP, b=BP), t.format(w=64, d=ZP, a=XP, b=YP)] +
            nan_fix(g, [(RP, AP, BP), (ZP, XP, YP)], 64) + g.w128(R, Z) + g.next(), slots=2)
    FCMP = {"EQ": "eq", "NE": "neq", "LT": "lt", "GT": "gt", "LE": "le", "GE": "ge"}
    for nm, c in FCMP.items():
        add("F32_" + nm, ["F32_" + nm], lambda g, c=c: [
            "v_cmp_%s_f32_e64 vcc, %s, %s" % (c, A[0], B[0])] + g.bool_result() + g.next())
        add("F64_" + nm, ["F64_" + nm], lambda g, c=c: [
            "v_cmp_%s_f64_e64 vcc, %s, %s" % (c, AP, BP)] + g.bool_result() + g.next())
        add("V_F32X4_" + nm, ["V_F32X4_" + nm], lambda g, c=c: hi_reads(g, [(AADDR, XP), (BADDR, YP)]) + [
            "v_cmp_%s_f32_e64 vcc, %s, %s" % (c, A[0], B[0]), "v_cndmask_b32_e64 %s, 0, -1, vcc" % R[0],
            "v_cmp_%s_f32_e64 vcc, %s, %s" % (c, A[1], B[1]), "v_cndmask_b32_e64 %s, 0, -1, vcc" % R[1],
            "v_cmp_%s_f32_e64 vcc, %s, %s" % (c, X[0], Y[0]), "v_cndmask_b32_e64 %s, 0, -1, vcc" % Z[0],
            "v_cmp_%s_f32_e64 vcc, %s, %s" % (c, X[1], Y[1]), "v_cndmask_b32_e64 %s, 0, -1, vcc" % Z[1]] +
            g.w128(R, Z) + g.next())
        add("V_F64X2_" + nm, ["V_F64X2_" + nm], lambda g, c=c: hi_reads(g, [(AADDR, XP), (BADDR, YP)]) + [
            "v_cmp_%s_f64_e64 vcc, %s, %s" % (c, AP, BP), "v_cndmask_b32_e64 %s, 0, -1, vcc" % R[0],
            "v_mov_b32 %s, %s" % (R[1], R[0]),
            "v_cmp_%s_f64_e64 vcc, %s, %s" % (c, XP, YP), "v_cndmask_b32_e64 %s, 0, -1, vcc" % Z[0],
            "v_mov_b32 %s, %s" % (Z[1], Z[0])] + g.w128(R, Z) + g.next())
    add("F32_ABS", ["F32_ABS"], lambda g: ["v_and_b32_e32 %s, 0x7fffffff, %s" % (R[0], A[0])] +
        g.w32() + g.next())
    add("F32_NEG", ["F32_NEG"], lambda g: ["v_xor_b32_e32 %s, 0x80000000, %s" % (R[0], A[0])] +
        g.w32() + g.next())
    add("F64_ABS", ["F64_ABS"], lambda g: ["v_and_b32_e32 %s, 0x7fffffff, %s" % (R[1], A[1])] +
        g.w64(A[0], R[1]) + g.next())
    add("F64_NEG", ["F64_NEG"], lambda g: ["v_xor_b32_e32 %s, 0x80000000, %s" % (R[1], A[1])] +
        g.w64(A[0], R[1]) + g.next())
    # (VOP3 takes no literal on gfx9: the mask goes through an SGPR)
    add("F32_COPYSIGN", ["F32_COPYSIGN"], lambda g: ["s_mov_b32 s68, 0x7fffffff",
        "v_bfi_b32 %s, s68, %s, %s" % (R[0], A[0], B[0])] + g.w32() + g.next())
    add("F64_COPYSIGN", ["F64_COPYSIGN"], lambda g: ["s_mov_b32 s68, 0x7fffffff",
        "v_bfi_b32 %s, s68, %s, %s" % (R[1], A[1], B[1])] + g.w64(A[0], R[1]) + g.next())
    add("F64_CONVERT_I32_S", ["F64_CONVERT_I32_S"], lambda g: [
        "v_cvt_f64_i32_e32 %s, %s" % (RP, A[0])] + g.w64() + g.next())
    add("F64_CONVERT_I32_U", ["F64_CONVERT_I32_U"], lambda g: [
        "v_cvt_f64_u32_e32 %s, %s" % (RP, A[0])] + g.w64() + g.next())
    add("F32_CONVERT_I32_S", ["F32_CONVERT_I32_S"], lambda g: [
        "v_cvt_f32_i32_e32 %s, %s" % (R[0], A[0])] + g.w32() + g.next())
    add("F32_CONVERT_I32_U", ["F32_CONVERT_I32_U"], lambda g: [
        "v_cvt_f32_u32_e32 %s, %s" % (R[0], A[0])] + g.w32() + g.next())
    add("F64_PROMOTE_F32", ["F64_PROMOTE_F32"], lambda g: [
        "v_cvt_f64_f32_e32 %s, %s" % (RP, A[0])] + nan_exit(g, [RP], 64) + g.w64() + g.next())
    add("F32_DEMOTE_F64", ["F32_DEMOTE_F64"], lambda g: [
        "v_cvt_f32_f64_e32 %s, %s" % (R[0], AP)] + nan_exit(g, [R[0]], 32) + g.w32() + g.next())
    # ---- SIMD128 data movement / integer lanes (4 cells; cells +2, +3 read here)
    add("MOV128", ["MOV128"], lambda g: hi_reads(g, [(AADDR, XP)]) + g.w128(A, X) + g.next())
    add("V_SPLAT32", ["V_I32X4_SPLAT", "V_F32X4_SPLAT"], lambda g: g.w128((A[0], A[0]), (A[0], A[0])) + g.next())
    add("V_SPLAT64", ["V_I64X2_SPLAT", "V_F64X2_SPLAT"], lambda g: g.w128(A, A) + g.next())
    # i64x2/f64x2.replace_lane: w7 = the lane (tc.cpp); lane 0 -> (b, a.hi), 1 -> (a.lo, b)
    add("V_REPLACE64", ["V_REPLACE64"], lambda g: hi_reads(g, [(AADDR, XP)]) + [
        "s_cmp_eq_u32 %s, 0" % g.x(7),
        "s_cselect_b64 %s, exec, 0" % T2,
        "v_cndmask_b32_e64 %s, %s, %s, %s" % (R[0], A[0], B[0], T2),
        "v_cndmask_b32_e64 %s, %s, %s, %s" % (R[1], A[1], B[1], T2),
        "v_cndmask_b32_e64 %s, %s, %s, %s" % (Z[0], B[0], X[0], T2),
        "v_cndmask_b32_e64 %s, %s, %s, %s" % (Z[1], B[1], X[1], T2)] + g.w128(R, Z) + g.next())
    VBIT = {"V_AND": "v_and_b32_e32 {d}, {a}, {b}", "V_OR": "v_or_b32_e32 {d}, {a}, {b}",
            "V_XOR": "v_xor_b32_e32 {d}, {a}, {b}", "V_I32X4_ADD": "v_add_u32_e32 {d}, {a}, {b}",
            "V_I32X4_SUB": "v_sub_u32_e32 {d}, {a}, {b}", "V_I32X4_MUL": "v_mul_lo_u32 {d}, {a}, {b}"}
    for nm, t in VBIT.items():
        add(nm, [nm], lambda g, t=t: hi_reads(g, [(AADDR, XP), (BADDR, YP)]) + [
            t.format(d=R[0], a=A[0], b=B[0]), t.format(d=R[1], a=A[1], b=B[1]),
            t.format(d=Z[0], a=X[0], b=Y[0]), t.format(d=Z[1], a=X[1], b=Y[1])] + g.w128(R, Z) + g.next())
    add("V_I64X2_ADD", ["V_I64X2_ADD"], lambda g: hi_reads(g, [(AADDR, XP), (BADDR, YP)]) + [
        "v_lshl_add_u64 %s, %s, 0, %s" % (RP, AP, BP), "v_lshl_add_u64 %s, %s, 0, %s" % (ZP, XP, YP)] +
        g.w128(R, Z) + g.next())
    add("V_I64X2_SUB", ["V_I64X2_SUB"], lambda g: hi_reads(g, [(AADDR, XP), (BADDR, YP)]) + [
        "v_sub_co_u32_e64 %s, vcc, %s, %s" % (R[0], A[0], B[0]),
        "v_subb_co_u32_e64 %s, vcc, %s, %s, vcc" % (R[1], A[1], B[1]),
        "v_sub_co_u32_e64 %s, vcc, %s, %s" % (Z[0], X[0], Y[0]),
        "v_subb_co_u32_e64 %s, vcc, %s, %s, vcc" % (Z[1], X[1], Y[1])] + g.w128(R, Z) + g.next())
    add("V_I64X2_EQ", ["V_I64X2_EQ"], lambda g: hi_reads(g, [(AADDR, XP), (BADDR, YP)]) + [
        "v_cmp_eq_u64_e64 vcc, %s, %s" % (AP, BP), "v_cndmask_b32_e64 %s, 0, -1, vcc" % R[0],
        "v_mov_b32 %s, %s" % (R[1], R[0]),
        "v_cmp_eq_u64_e64 vcc, %s, %s" % (XP, YP), "v_cndmask_b32_e64 %s, 0, -1, vcc" % Z[0],
        "v_mov_b32 %s, %s" % (Z[1], Z[0])] + g.w128(R, Z) + g.next())
    add("V_ANY_TRUE", ["V_ANY_TRUE"], lambda g: hi_reads(g, [(AADDR, XP)]) + [
        "v_or3_b32 %s, %s, %s, %s" % (R[0], A[0], A[1], X[0]),
        "v_or_b32_e32 %s, %s, %s" % (R[0], R[0], X[1]),
        "v_cmp_ne_u32_e64 vcc, 0, %s" % R[0]] + g.bool_result() + g.next())
    add("V_I32X4_BITMASK", ["V_I32X4_BITMASK"], lambda g: hi_reads(g, [(AADDR, XP)]) + [
        "v_lshrrev_b32_e32 %s, 31, %s" % (R[0], A[0]),
        "v_lshrrev_b32_e32 %s, 31, %s" % (R[1], A[1]),
        "v_lshl_or_b32 %s, %s, 1, %s" % (R[0], R[1], R[0]),
        "v_lshrrev_b32_e32 %s, 31, %s" % (R[1], X[0]),
        "v_lshl_or_b32 %s, %s, 2, %s" % (R[0], R[1], R[0]),
        "v_lshrrev_b32_e32 %s, 31, %s" % (R[1], X[1]),
        "v_lshl_or_b32 %s, %s, 3, %s" % (R[0], R[1], R[0])] + g.w32() + g.next())
    add("CALL", ["CALL"], call_body, slots=2)
    add("RET", ["RET"], ret_body, slots=2)
    add("POST_CALL", ["POST_CALL"], post_call_body, slots=2)
    add("TAIL_CALL", ["TAIL_CALL"], tail_call_body, slots=2)
    add("I32_CLZ", ["I32_CLZ"], lambda g: [
        "v_ffbh_u32_e32 %s, %s" % (X[0], A[0]),
        "v_min_u32_e32 %s, 32, %s" % (R[0], X[0])] + g.w32() + g.next())
    add("I32_CTZ", ["I32_CTZ"], lambda g: [
        "v_ffbl_b32_e32 %s, %s" % (X[0], A[0]),
        "v_min_u32_e32 %s, 32, %s" % (R[0], X[0])] + g.w32() + g.next())
    add("I32_POPCNT", ["I32_POPCNT"], lambda g: [
        "v_bcnt_u32_b32 %s, %s, 0" % (R[0], A[0])] + g.w32() + g.next())
    add("I32_EXT8S", ["I32_EXT8S"], lambda g: ["v_bfe_i32 %s, %s, 0, 8" % (R[0], A[0])] +
        g.w32() + g.next())
    add("I32_EXT16S", ["I32_EXT16S"], lambda g: ["v_bfe_i32 %s, %s, 0, 16" % (R[0], A[0])] +
        g.w32() + g.next())
    # ---- i64 (operands A = a.lo/a.hi; *_I: imm sign-extended from w4)
    def imm64(g):   # VGPRs, so VOP3 ops keep to gfx9's one-SGPR constant-bus limit
        return ["v_mov_b32 %s, %s" % (Z[0], g.x(4)), "v_ashrrev_i32_e32 %s, 31, %s" % (Z[1], Z[0])]

    def i64_bin(name, body):   # body(g, b_lo, b_hi, b_pair) -> lines
        add("I64_" + name, ["I64_" + name],
            lambda g: body(g, B[0], B[1], BP) + g.w64() + g.next())
        add("I64_%s_I" % name, ["I64_%s_I" % name],
            lambda g: imm64(g) + body(g, Z[0], Z[1], ZP) + g.w64() + g.next())

    i64_bin("ADD", lambda g, lo, hi, p: ["v_lshl_add_u64 %s, %s, 0, %s" % (RP, AP, p)])
    i64_bin("SUB", lambda g, lo, hi, p: ["v_sub_co_u32_e64 %s, vcc, %s, %s" % (R[0], A[0], lo),
                                         "v_subb_co_u32_e64 %s, vcc, %s, %s, vcc" % (R[1], A[1], hi)])
    for nm, ins in (("AND", "v_and_b32_e64"), ("OR", "v_or_b32_e64"), ("XOR", "v_xor_b32_e64")):
        i64_bin(nm, lambda g, lo, hi, p, ins=ins: ["%s %s, %s, %s" % (ins, R[0], A[0], lo),
                                                   "%s %s, %s, %s" % (ins, R[1], A[1], hi)])
    i64_bin("MUL", lambda g, lo, hi, p: [
        "v_mul_hi_u32 %s, %s, %s" % (X[0], A[0], lo),
        "v_mul_lo_u32 %s, %s, %s" % (X[1], A[0], hi),
        "v_mul_lo_u32 %s, %s, %s" % (Y[0], A[1], lo),
        "v_mul_lo_u32 %s, %s, %s" % (R[0], A[0], lo),
        "v_add3_u32 %s, %s, %s, %s" % (R[1], X[0], X[1], Y[0])])
    i64_bin("SHL", lambda g, lo, hi, p: ["v_lshlrev_b64 %s, %s, %s" % (RP, lo, AP)])
    i64_bin("SHR_S", lambda g, lo, hi, p: ["v_ashrrev_i64 %s, %s, %s" % (RP, lo, AP)])
    i64_bin("SHR_U", lambda g, lo, hi, p: ["v_lshrrev_b64 %s, %s, %s" % (RP, lo, AP)])
    i64_bin("ROTL", lambda g, lo, hi, p: [
        "v_sub_u32_e64 %s, 0, %s" % (Y[0], lo),
        "v_lshlrev_b64 %s, %s, %s" % (XP, lo, AP),
        "v_lshrrev_b64 %s, %s, %s" % (RP, Y[0], AP),
        "v_or_b32_e32 %s, %s, %s" % (R[0], R[0], X[0]),
        "v_or_b32_e32 %s, %s, %s" % (R[1], R[1], X[1])])
    i64_bin("ROTR", lambda g, lo, hi, p: [
        "v_sub_u32_e64 %s, 0, %s" % (Y[0], lo),
        "v_lshrrev_b64 %s, %s, %s" % (XP, lo, AP),
        "v_lshlrev_b64 %s, %s, %s" % (RP, Y[0], AP),
        "v_or_b32_e32 %s, %s, %s" % (R[0], R[0], X[0]),
        "v_or_b32_e32 %s, %s, %s" % (R[1], R[1], X[1])])
    for c, k in CMP.items():
        k64 = k + "64"
        add("I64_" + c, ["I64_" + c], lambda g, k64=k64: [
            "v_cmp_%s_e64 vcc, %s, %s" % (k64, AP, BP)] + g.bool_result() + g.next())
        add("I64_%s_I" % c, ["I64_%s_I" % c], lambda g, k64=k64: imm64(g) + [
            "v_cmp_%s_e64 vcc, %s, %s" % (k64, AP, ZP)] + g.bool_result() + g.next())
    add("I64_EQZ", ["I64_EQZ"], lambda g: ["v_cmp_eq_u64_e64 vcc, 0, %s" % AP] +
        g.bool_result() + g.next())
    add("I64_EXTEND_I32_S", ["I64_EXTEND_I32_S", "I64_EXT32S"], lambda g: [
        "v_ashrrev_i32_e32 %s, 31, %s" % (R[1], A[0])] + g.w64(A[0], R[1]) + g.next())
    add("I64_EXTEND_I32_U", ["I64_EXTEND_I32_U"], lambda g: [
        "v_mov_b32 %s, 0" % R[1]] + g.w64(A[0], R[1]) + g.next())
    add("I64_EXT8S", ["I64_EXT8S"], lambda g: [
        "v_bfe_i32 %s, %s, 0, 8" % (R[0], A[0]),
        "v_ashrrev_i32_e32 %s, 31, %s" % (R[1], R[0])] + g.w64() + g.next())
    add("I64_EXT16S", ["I64_EXT16S"], lambda g: [
        "v_bfe_i32 %s, %s, 0, 16" % (R[0], A[0]),
        "v_ashrrev_i32_e32 %s, 31, %s" % (R[1], R[0])] + g.w64() + g.next())

    # ---- linear memory. w4 = offset, w7 = offset + n - 1 (< 2^32, else the op is cold).
    # In bounds  <=> no carry in a + (offset+n-1)  and  (last byte >> 16) < pages;
    # natural alignment of ea (4 for n >= 4) <=> (last byte & m) == m.
    def mem_check(g, n):
        out = ["v_add_co_u32_e64 %s, %s, %s, %s" % (X[0], T2, A[0], g.x(7)),   # last byte
               "v_lshrrev_b32_e32 %s, 16, %s" % (X[1], X[0]),
               "v_cmp_ge_u32_e64 vcc, %s, %s" % (X[1], PAGES),
               "s_or_b64 %s, %s, vcc" % (T2, T2)]
        m = 3 if n >= 4 else n - 1
        if m:
            out += ["v_and_b32_e32 %s, %d, %s" % (Y[0], m, X[0]),
                    "v_cmp_ne_u32_e64 vcc, %d, %s" % (m, Y[0]),
                    "s_or_b64 %s, %s, vcc" % (T2, T2)]
        out += ["s_and_b64 %s, %s, exec" % (T2, T2), "s_cbranch_scc1 %s" % g.xh(),
                "v_add_u32_e64 %s, %s, %s" % (Y[0], A[0], g.x(4))] + gaddr(XP, Y[0])
        return out

    # address of byte `ea` of this lane's memory: MEM (wave base + lane granule) +
    # (ea >> (2+g)) granule rows of 256 << g bytes + the byte within the granule
    def gaddr(dst, ea):
        return ["v_lshrrev_b32_e32 %s, %s, %s" % (W[0], MSH1, ea),
                "v_lshlrev_b64 %s, %s, %s" % (dst, MSH2, WP),  # W[1] is always 0
                "v_lshl_add_u64 %s, %s, 0, %s" % (dst, dst, MEM),
                "v_bfe_u32 %s, %s, 0, %s" % (W[0], ea, MSH1),
                "v_lshl_add_u64 %s, %s, 0, %s" % (dst, WP, dst)]

    LOADS = {   # name -> (bytes, load instr, result width, sign-extend high word)
        "LD32": (4, "global_load_dword", 32, None),
        "LD8U32": (1, "global_load_ubyte", 32, None),
        "LD8S32": (1, "global_load_sbyte", 32, None),
        "LD16U32": (2, "global_load_ushort", 32, None),
        "LD16S32": (2, "global_load_sshort", 32, None),
        "LD32U64": (4, "global_load_dword", 64, "zero"),
        "LD32S64": (4, "global_load_dword", 64, "sign"),
        "LD8U64": (1, "global_load_ubyte", 64, "zero"),
        "LD8S64": (1, "global_load_sbyte", 64, "sign"),
        "LD16U64": (2, "global_load_ushort", 64, "zero"),
        "LD16S64": (2, "global_load_sshort", 64, "sign"),
    }
    for nm, (n, ins, width, ext) in LOADS.items():
        def body(g, n=n, ins=ins, width=width, ext=ext):
            out = mem_check(g, n) + ["%s %s, %s, off" % (ins, R[0], XP), "s_waitcnt vmcnt(0)"]
            if width == 32:
                return out + g.w32() + g.next()
            hi = "v_mov_b32 %s, 0" % R[1] if ext == "zero" else \
                "v_ashrrev_i32_e32 %s, 31, %s" % (R[1], R[0])
            return out + [hi] + g.w64() + g.next()
        add(nm, [nm], body)
    def word2():   # ZP = address of the second word (ea + 4: maybe another granule)
        return ["v_add_u32_e32 %s, 4, %s" % (Y[1], Y[0])] + gaddr(ZP, Y[1])
    add("LD64", ["LD64"], lambda g: mem_check(g, 8) + word2() + [
        "global_load_dword %s, %s, off" % (R[0], XP),
        "global_load_dword %s, %s, off" % (R[1], ZP),
        "s_waitcnt vmcnt(0)"] + g.w64() + g.next())
    STORES = {"ST8": (1, "global_store_byte"), "ST16": (2, "global_store_short"),
              "ST32": (4, "global_store_dword")}
    def mark(n):   # HWM = max(HWM, ea + n), saturating (Y0 = ea from mem_check)
        return ["v_add_u32_e64 %s, %s, %d clamp" % (Y[1], Y[0], n),
                "v_max_u32_e32 %s, %s, %s" % (HWM, HWM, Y[1])]
    for nm, (n, ins) in STORES.items():
        add(nm, [nm], lambda g, n=n, ins=ins: mem_check(g, n) + [
            "%s %s, %s, off" % (ins, XP, B[0])] + mark(n) + g.next())
    add("ST64", ["ST64"], lambda g: mem_check(g, 8) + word2() + [
        "global_store_dword %s, %s, off" % (XP, B[0]),
        "global_store_dword %s, %s, off" % (ZP, B[1])] + mark(8) + g.next())
    # ---- memories past the first (MultiMemories; XLD / XST with the memory-0 op in D,
    # jit.cpp emit_xmem). V blob only (the LDS blob leaves them to the C++ step). The
    # translator (tc.cpp) picks the slot by that op and sets: w1 = the address cell, w2 =
    # (XLD) memory k's declared minimum in pages / (XST) the value cell, w3 = (XLD) the
    # result cell / (XST) the minimum, w4 = offset, w5 = memory k's word offset in a lane's
    # block (xinfo, a multiple of 16384) | the granule log g, w7 = offset + n - 1. Bounds
    # against the minimum (every lane's memory k has at least that many pages; past it the
    # C++ step decides), alignment as mem_check; the wave's block is s[98:99] (the kernel
    # sets it at every core call), the lane's byte ea at block + w5 / 32 * 32 * 256 +
    # (lane << (2 + g)) + (ea >> (2 + g) << (8 + g)) + (ea & (4 << g) - 1).
    def xmem_addr(g, n, minp):
        out = ["v_add_co_u32_e64 %s, %s, %s, %s" % (X[0], T2, A[0], g.x(7)),   # last byte
               "v_lshrrev_b32_e32 %s, 16, %s" % (X[1], X[0]),
               "v_cmp_le_u32_e64 vcc, %s, %s" % (minp, X[1]),
               "s_or_b64 %s, %s, vcc" % (T2, T2)]
        m = 3 if n >= 4 else n - 1
        if m:
            out += ["v_and_b32_e32 %s, %d, %s" % (Y[0], m, X[0]),
                    "v_cmp_ne_u32_e64 vcc, %d, %s" % (m, Y[0]),
                    "s_or_b64 %s, %s, vcc" % (T2, T2)]
        out += ["s_and_b64 %s, %s, exec" % (T2, T2), "s_cbranch_scc1 %s" % g.xh(),
                "v_add_u32_e64 %s, %s, %s" % (Y[0], A[0], g.x(4)),   # ea
                "s_and_b32 s68, %s, 31" % g.x(5),                     # g
                "s_andn2_b32 s69, %s, 31" % g.x(5),                   # word offset
                "s_lshl_b32 s74, s69, 8", "s_lshr_b32 s75, s69, 24",  # (T2 is free again)
                "s_add_u32 s74, s74, s98", "s_addc_u32 s75, s75, s99",
                "s_add_u32 s69, s68, 2",
                "s_add_u32 s68, s68, 8",
                "v_mbcnt_lo_u32_b32 %s, -1, 0" % W[0],
                "v_mbcnt_hi_u32_b32 %s, -1, %s" % (W[0], W[0]),
                "v_lshlrev_b32_e64 %s, s69, %s" % (W[0], W[0]),
                "v_lshl_add_u64 %s, %s, 0, s[74:75]" % (ZP, WP)]      # ZP = the lane's granule 0
        def at(dst, ea):
            return ["v_lshrrev_b32_e64 %s, s69, %s" % (W[0], ea),
                    "v_lshlrev_b64 %s, s68, %s" % (dst, WP),
                    "v_lshl_add_u64 %s, %s, 0, %s" % (dst, dst, ZP),
                    "v_bfe_u32 %s, %s, 0, s69" % (W[0], ea),
                    "v_lshl_add_u64 %s, %s, 0, %s" % (dst, WP, dst)]
        return out + at(XP, Y[0])

    def x_word2(g):   # XP = the second word's address (ea + 4: maybe the next granule), once
        # the first word's access has gone out (a memory instruction reads XP at issue)
        return ["v_add_u32_e32 %s, 4, %s" % (Y[1], Y[0]),
                "v_lshrrev_b32_e64 %s, s69, %s" % (W[0], Y[1]),
                "v_lshlrev_b64 %s, s68, %s" % (XP, WP),
                "v_lshl_add_u64 %s, %s, 0, %s" % (XP, XP, ZP),
                "v_bfe_u32 %s, %s, 0, s69" % (W[0], Y[1]),
                "v_lshl_add_u64 %s, %s, 0, %s" % (XP, WP, XP)]

    def x_exit(g):
        return g.exit_here()
    for nm, (n, ins, width, ext) in LOADS.items():
        def xbody(g, n=n, ins=ins, width=width, ext=ext):
            if not g.vf:
                return x_exit(g)
            out = xmem_addr(g, n, g.x(2)) + ["%s %s, %s, off" % (ins, R[0], XP), "s_waitcnt vmcnt(0)"]
            if width == 32:
                return out + g.w32() + g.next()
            hi = "v_mov_b32 %s, 0" % R[1] if ext == "zero" else "v_ashrrev_i32_e32 %s, 31, %s" % (R[1], R[0])
            return out + [hi] + g.w64() + g.next()
        add("XLD_" + nm, [], xbody)
    add("XLD_LD64", [], lambda g: x_exit(g) if not g.vf else xmem_addr(g, 8, g.x(2)) + [
        "global_load_dword %s, %s, off" % (R[0], XP)] + x_word2(g) + [
        "global_load_dword %s, %s, off" % (R[1], XP),
        "s_waitcnt vmcnt(0)"] + g.w64() + g.next(), slots=2)
    for nm, (n, ins) in STORES.items():
        add("XST_" + nm, [], lambda g, n=n, ins=ins: x_exit(g) if not g.vf else xmem_addr(g, n, g.x(3)) + [
            "%s %s, %s, off" % (ins, XP, B[0])] + g.next())
    add("XST_ST64", [], lambda g: x_exit(g) if not g.vf else xmem_addr(g, 8, g.x(3)) + [
        "global_store_dword %s, %s, off" % (XP, B[0])] + x_word2(g) + [
        "global_store_dword %s, %s, off" % (XP, B[1])] + g.next(), slots=2)
    # ---- compiled blocks (jit.cpp): a straight-line run of instructions compiled for
    # this module, entered here. Fields: w1/w2 = the block's code address, w5 = (run
    # length - 1) * 32. The block reloads both banks for the instruction after the run
    # and dispatches it itself (bank A), or leaves through slot 0 (xh at +0, xs at
    # +JIT_XS). Diverged mode: a run that would pass the lowest waiting pc is left to
    # the C++ step (it never does in practice: runs hold no jump target).
    def jit_body(g):
        if not g.vf:
            return g.exit_here()
        out = [SELF]
        if g.mode == "D":
            out += ["s_add_u32 s68, %s, %s" % (PCOFF, g.x(5)),
                    "s_cmp_ge_u32 s68, %s" % OTHER, "s_cbranch_scc1 %s" % g.xh()]
        return out + ["s_mov_b32 s68, %s" % g.x(1), "s_mov_b32 s69, %s" % g.x(2),
                      "s_setpc_b64 s[68:69]"]
    add("JIT", [], jit_body)
    # ---- fused pairs (V blob, converged mode): the instruction at pc (a fall-through
    # op) and the one at pc + 1 in one handler, saving a dispatch. tc.cpp picks the slot
    # from the two instructions' own slots (tc_pair_slot); each half reads its own
    # TInstr (pc's in this bank, pc + 1's in the other), so either may exit before its
    # effect exactly as alone. Elsewhere (LDS blob, diverged mode) the slot runs pc alone.
    # Pairs: the most frequent fall-through pairs of the BASELINE workloads
    # (tools/pair_hist.py).
    body_of = {nm: b for nm, _, b in S if b is not None}

    def tuple_spec(fs):
        def body(g):
            if not g.vf or g.mode == "D":
                return fs[0](g)
            out, bank = [SELF], g.bank
            for k, f in enumerate(fs):
                gk = Gen(g.mode, bank, True)
                gk.glue = k + 1 < len(fs)   # all but the last hand over to the next
                gk.stubs = g.bank           # stay within branch range of this bank's stubs
                out += vproc(gk, f(gk))
                bank = gk.other
            return out
        return body

    for tup in TUPLES:
        nm = "P_" + "__".join(tup)
        S.append((nm, [], tuple_spec([body_of[x] for x in tup])))
        # FP add/sub/mul carry their in-place NaN fix: one more slot each
        nfix = sum(1 for x in tup if x.split("_")[0] in ("F32", "F64", "V")
                   and x.split("_")[-1] in ("ADD", "SUB", "MUL") and "F" in x.split("_")[-2])
        for k in range(1, max(2, len(tup)) + nfix):
            S.append(("%s+%d" % (nm, k), [], None))
    return S


# fused tuples: every op but the last falls through; longest match first (tc.cpp)
ARX = ("I32_ADD3_XROTR_I", "I32_ADD_XROTR_I")
TUPLES = [ARX * 4, ARX[::-1] * 4, ARX * 2, ARX[::-1] * 2]
TUPLES_PAIRS = [
    ("I32_ADD3_XROTR_I", "I32_ADD_XROTR_I"), ("I32_ADD_XROTR_I", "I32_ADD3_XROTR_I"),
    ("LD32", "LD32"), ("I32_XOR", "ST32"), ("ST32", "I32_XOR"), ("I64_SHR_U_I", "I64_XOR"),
    ("I64_XOR", "CONST64"), ("CONST64", "I64_MUL"), ("I64_MUL", "I64_SHR_U_I"),
    ("CONST32", "CONST32"), ("CONST64", "I64_ADD"), ("I64_ADD", "MOV64"),
    ("I32_SUB_I", "LD32"), ("LD32", "BR_GT_S"), ("I32_ADD_I", "LD32"), ("LD32", "BR_LT_S"),
    ("LD32", "ST32"), ("ST32", "ST32"), ("ST32", "JMP"), ("I32_SHL_I", "I32_XOR"),
    ("I32_ADD_I", "JMP"), ("I64_LE_U_I", "BR_UNLESS"), ("I64_AND_I", "I32_ADD_I"),
    ("I32_ADD_I", "CONST32"), ("CONST32", "JMP"), ("I64_SHR_U_I", "I32_ADD_I"),
    ("I64_MUL_I", "I64_ADD_I"), ("I64_ADD_I", "I64_GT_U"), ("I64_GT_U", "BR_UNLESS"),
    ("MOV64", "I32_ADD_I"), ("CONST64", "V_SPLAT64"), ("V_F64X2_MUL", "V_F64X2_ADD"),
    ("I32_SHL_I", "I32_ADD"), ("V_F64X2_MUL", "V_F64X2_MUL"), ("V_F64X2_ADD", "CONST64"),
    ("V_SPLAT64", "V_F64X2_LE"), ("V_F64X2_LE", "V_ANY_TRUE"), ("V_ANY_TRUE", "BR_UNLESS"),
    ("V_I64X2_SUB", "V_F64X2_MUL"), ("V_F64X2_MUL", "CONST64"), ("V_SPLAT64", "V_F64X2_MUL"),
]
TUPLES += TUPLES_PAIRS


SPECIAL_REMAP = {   # DBC op -> (slot op, immediate transform) applied by the translator
    "I32_ROTL_I": ("I32_ROTR_I", "neg32"),
    "I32_XOR_ROTL_I": ("I32_XOR_ROTR_I", "neg32"),
}


def vfuse_src(body):
    """V-frame peephole: the last operand fetched by an index-mode move that only feeds
    the next instruction's first source is read there directly as an indexed source."""
    out = list(body)
    i = 0
    while i + 3 < len(out):
        m = re.match(r"v_mov_b32 (v\d+), v%d$" % VB, out[i + 1])
        if (m and out[i].startswith(("s_set_gpr_idx_idx", "s_set_gpr_idx_on")) and
                (out[i].startswith("s_set_gpr_idx_idx") or out[i].endswith("gpr_idx(SRC0)")) and
                out[i + 2] == "s_set_gpr_idx_off"):
            q = m.group(1)
            mi = re.match(r"(v_\w+) ([\w\[\]:]+), %s(, .*)?$" % q, out[i + 3])
            rest = (mi.group(3) or "") if mi else ""
            if (mi and not mi.group(1).startswith(("v_readfirstlane", "v_mov")) and
                    not re.search(r"\b%s\b" % q, rest) and "v[" not in rest and
                    "v[" not in mi.group(2) and
                    not any(re.search(r"\b%s\b" % q, ln) for ln in out[i + 4:])):
                out[i + 1:i + 4] = ["%s %s, v%d%s" % (mi.group(1), mi.group(2), VB, rest),
                                    "s_set_gpr_idx_off"]
        i += 1
    return out


def vproc(g, b):
    """V-blob processing of one handler body: operand prologue and peepholes."""
    if b and b[0] == SELF:   # reads its operands itself
        body = b[1:]
    else:
        body = vfuse_src(vfuse(g.vprologue(b) + b))
    # an index-off directly followed by an index-on is redundant
    return [ln for k, ln in enumerate(body) if not (
        ln == "s_set_gpr_idx_off" and k + 1 < len(body) and body[k + 1].startswith("s_set_gpr_idx_on"))]


def vfuse(body):
    """V-frame peephole: a VALU op computing R0 that is then only moved into an indexed
    frame cell computes straight into that cell (its sources are plain VGPRs, so DST
    indexing touches only the result), and an index-off right before an index-on goes."""
    r0 = R[0]
    out = list(body)
    i = 0
    while i + 3 < len(out):
        ins = out[i]
        m = re.match(r"(v_\w+) %s, (.*)$" % r0, ins)
        if (m and not m.group(1).startswith(("v_cmp", "v_readfirstlane", "v_mov_b32")) and
                not re.search(r"\b%s\b" % r0, m.group(2)) and "v[" not in m.group(2) and
                out[i + 1].startswith("s_set_gpr_idx_on") and out[i + 1].endswith("gpr_idx(DST)") and
                out[i + 2] == "v_mov_b32 v%d, %s" % (VB, r0) and out[i + 3] == "s_set_gpr_idx_off" and
                not any(re.search(r"\b%s\b|v\[114:115\]" % r0, ln) for ln in out[i + 4:])):
            out[i:i + 4] = [out[i + 1], "%s v%d, %s" % (m.group(1), VB, m.group(2)), "s_set_gpr_idx_off"]
            if i and out[i - 1] == "s_set_gpr_idx_off":
                del out[i - 1]
                i -= 1
        i += 1
    return out


def blob(S, names, vf):
    """Assembly lines of one handler blob: LDS frames (vf False, entry wb_tc_entry) or
    V frames (vf True, entry wb_vf_entry)."""
    pre = "Lvf" if vf else "Ltc"
    nslots = len(names)
    bank_bytes = nslots * SLOT
    L = []
    e = L.append
    e(".text")
    e(".p2align 8")
    # ------------------------------------------------------------- entry
    # in: CODE, PCOFF (pc*32 of the first instruction), OTHER, LOW, LIM, CNT=0, RET,
    #     FR, PAGES, MEM (V frames also VSYNC).  EXEC = the active lanes.
    e("%s:" % ("wb_vf_entry" if vf else "wb_tc_entry"))
    e("s_getpc_b64 s[70:71]")
    e("%s_pc0:" % pre)
    e("s_add_u32 s70, s70, %s_banks - %s_pc0" % (pre, pre))
    e("s_addc_u32 s71, s71, 0")
    e("s_cmp_eq_u32 %s, -1" % LOW)                    # no lane waiting: banks 0/1
    e("s_cselect_b32 %s, 0, %d" % (T[0], 2 * bank_bytes))
    e("s_add_u32 s70, s70, %s" % T[0])
    e("s_addc_u32 s71, s71, 0")
    e("s_add_u32 s72, s70, %d" % bank_bytes)
    e("s_addc_u32 s73, s71, 0")
    e("v_mov_b32 %s, 0" % W[1])
    e("s_load_dwordx8 %s, %s, %s" % (sbank("A"), CODE, PCOFF))
    e("s_load_dwordx8 %s, %s, %s offset:0x20" % (sbank("B"), CODE, PCOFF))
    g0 = Gen("C", "B", vf)
    if vf:
        # frame LDS -> VGPRs: jump into an unrolled run of ds_reads (cells VMAX-1 .. 0;
        # VSYNC = (VMAX - cells) * 8 skips the ones past the frame)
        e("s_getpc_b64 s[68:69]")
        e("Lvf_si_pc:")
        e("s_add_u32 s68, s68, Lvf_si_base - Lvf_si_pc")
        e("s_addc_u32 s69, s69, 0")
        e("s_add_u32 s68, s68, %s" % VSYNC)
        e("s_addc_u32 s69, s69, 0")
        e("s_setpc_b64 s[68:69]")
        e("Lvf_si_base:")
        for i in range(VMAX - 1, -1, -1):
            e("ds_read_b32 v%d, %s offset:%d" % (VB + i, FR, i * 256))
        e("s_waitcnt lgkmcnt(0)")
        # the frames of every lane in the core (ALL) are loaded; the group runs (SIMT
        # mode: batch_kernel.hip tc_run, jit.cpp Lsched; otherwise GROUP = ALL = EXEC)
        e("s_mov_b64 exec, %s" % GROUP)
        for ln in g0.dispatch("A"):
            e(ln)
    else:
        e("s_waitcnt lgkmcnt(0)")
        for ln in g0.issue_reads("A") + g0.dispatch("A"):
            e(ln)
    # ------------------------------------------------------------- banks
    e(".p2align 8")
    e("%s_banks:" % pre)
    for mode in ("C", "D"):
        for bank in ("A", "B"):
            for si, nm in enumerate(names):
                if si and S[si - 1][2] is None:
                    continue                       # covered by the multi-slot handler before
                span = 1
                while si + span < nslots and S[si + span - 1][2] is None:
                    span += 1
                g = Gen(mode, bank, vf)
                lab = "%s_%s%s_%d" % (pre, mode, bank, si)
                e(".p2align 8")
                e("%s:" % lab)
                if nm == "COLD":
                    # leave before this instruction (reason 0) / at PCOFF for the
                    # scheduler (reason 1); outstanding memory ops drained first
                    if vf:   # V frames go back to LDS first (Lvf_so_base)
                        body = []
                        for stub, why in ((g.xh(), 0), (g.xs(), 1)):
                            pcl = g.lab("so")
                            if why:   # compiled runs leave through slot 0 + JIT_XS
                                # (the xh stub is 56 bytes; checked below)
                                body += ["s_nop 0"] * ((JIT_XS - 56) // 4) + [
                                    ".if (. - %s) != %d" % (lab, JIT_XS),
                                    '.error "xs stub not at JIT_XS"', ".endif"]
                            # the group's lanes record where they stand (VPC) and what
                            # they retired since their last flush (VCNT), the group mask
                            # goes out in GROUP, then every lane in the core (ALL) stores
                            # its frame (Lvf_so_base + VSYNC: only the frame's cells)
                            body += ["%s:" % stub, "s_mov_b32 %s, %d" % (REASON, why),
                                     "s_getpc_b64 s[68:69]", "%s:" % pcl,
                                     "s_add_u32 s68, s68, Lvf_so_base - %s" % pcl,
                                     "s_addc_u32 s69, s69, 0",
                                     "s_add_u32 s68, s68, %s" % VSYNC, "s_addc_u32 s69, s69, 0",
                                     "v_lshrrev_b32_e64 %s, 5, %s" % (VPC, PCOFF),
                                     "v_add_u32_e32 %s, %s, %s" % (VCNT, CNT, VCNT),
                                     "s_mov_b64 %s, exec" % GROUP,
                                     "s_mov_b64 exec, %s" % ALL,
                                     "s_waitcnt vmcnt(0) lgkmcnt(0)", "s_setpc_b64 s[68:69]"]
                    else:
                        body = ["%s:" % g.xh(), "s_mov_b32 %s, 0" % REASON,
                                "s_waitcnt vmcnt(0) lgkmcnt(0)", "s_setpc_b64 %s" % RET,
                                "%s:" % g.xs(), "s_mov_b32 %s, 1" % REASON,
                                "s_waitcnt vmcnt(0) lgkmcnt(0)", "s_setpc_b64 %s" % RET]
                else:
                    spec = S[si - 1][2]
                    if vf:
                        body = vproc(g, spec(g))
                    else:
                        body = ["s_waitcnt lgkmcnt(0)"] + spec(g)
                for ln in body:
                    e(ln)
                e(".if (. - %s) > %d" % (lab, SLOT * span))
                e('.error "threaded-code handler %s exceeds its slot"' % nm)
                e(".endif")
                if span > 1:
                    e(".org %s + %d" % (lab, SLOT * span))
    e(".p2align 8")
    e("%s_banks_end:" % pre)
    if vf:
        # frame VGPRs -> LDS, then back to the kernel
        e("Lvf_so_base:")
        for i in range(VMAX - 1, -1, -1):
            e("ds_write_b32 %s, v%d offset:%d" % (FR, VB + i, i * 256))
        e("s_waitcnt lgkmcnt(0)")
        e("s_setpc_b64 %s" % RET)
    return L


def main():
    S = specs()
    names = ["COLD"] + [s[0] for s in S]
    nslots = len(names)
    for fname, vf, what in (("tc_blob.inc", False, "LDS frames"), ("tc_vblob.inc", True, "V frames")):
        with open(os.path.join(HERE, fname), "w") as f:
            f.write("// GENERATED by gen_tc.py -- do not edit. Handler blob of the threaded core (%s).\n" % what)
            for ln in blob(S, names, vf):
                f.write('"%s\\n"\n' % ln.replace('"', '\\"'))
    # ------------------------------------------------------------- slot map
    with open(os.path.join(HERE, "tc_slots.h"), "w") as f:
        f.write("// GENERATED by gen_tc.py -- do not edit. DBC op -> threaded-core slot.\n")
        f.write("#pragma once\n#include \"dbc.h\"\n\n")
        f.write("#define TC_SLOT_BYTES %d\n#define TC_NUM_SLOTS %d\n#define TC_VF_CELLS %d\n#define TC_JIT_XS %d\n"
                "#define TC_BANK_BYTES %d   // one bank; banks CA CB DA DB follow each other\n\n"
                % (SLOT, nslots, VMAX, JIT_XS, nslots * SLOT))
        for si, (nm, ops, body) in enumerate(S, start=1):
            if body is not None:
                f.write("#define TC_SLOT_%s %d\n" % (nm, si))
        f.write("\n// returns the handler slot (0 = no handler: the C++ step runs the op)\n")
        f.write("static inline int tc_slot(uint16_t op) {\n  switch (op) {\n")
        for si, (nm, ops, _) in enumerate(S, start=1):
            for op in ops:
                f.write("    case OP_%s: return %d;   // %s\n" % (op, si, nm))
        for op, (to, _) in SPECIAL_REMAP.items():
            f.write("    case OP_%s: return %d;   // via %s\n" % (op, names.index(to), to))
        f.write("    default: return 0;\n  }\n}\n")
        f.write("\n// fused tuple handler for the slots s[0..n) at pc.., longest first; *len = how\n"
                "// many instructions it covers; 0 = none (V blob)\n")
        f.write("static inline int tc_tuple_slot(const int *s, int n, int *len) {\n")
        tups = sorted([(nm[2:].split("__"), si) for si, (nm, ops, body) in enumerate(S, start=1)
                       if nm.startswith("P_") and body is not None], key=lambda t: -len(t[0]))
        for ops_, si in tups:
            cond = " && ".join("s[%d] == TC_SLOT_%s" % (k, o) for k, o in enumerate(ops_))
            f.write("  if (n >= %d && %s) { *len = %d; return %d; }\n" % (len(ops_), cond, len(ops_), si))
        f.write("  return 0;\n}\n")
    print("tc: %d slots, %d bytes per bank" % (nslots, nslots * SLOT), file=sys.stderr)


if __name__ == "__main__":
    main()
