/*
 * wasm_oracle.c -- TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's
 * interpreter path; see wasm_oracle.h for the file:line map and the parity pins.
 * Never linked into the product library; the GPU path fails loudly without its
 * HIP build instead of falling back here.
 *
 * Structure mirrors the reference on purpose (that is what makes it an oracle):
 *   - one flat Instr record per wasm instruction (include/ast/instruction.h:27-274),
 *   - loader-time JumpEnd/JumpElse/IsLast (lib/loader/ast/instruction.cpp:35-116),
 *   - validator-time Jump{EraseBegin,EraseEnd,PCOffset} and local StackOffset
 *     (lib/validator/formchecker.cpp:371-474, 655-673),
 *   - a value stack of untagged 16-byte slots + frame stack (include/runtime/stackmgr.h),
 *   - the dispatch loop that counts every dispatched instruction
 *     (lib/executor/engine/engine.cpp:1616-1637) plus the manual `else` count
 *     (lib/executor/engine/controlInstr.cpp:23-28).
 */
#define _GNU_SOURCE
#include "wasm_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ types */
typedef struct { uint64_t lo, hi; } Val;              /* ValVariant (types.h:84-88) */

enum { T_I32 = 0x7F, T_I64 = 0x7E, T_F32 = 0x7D, T_F64 = 0x7C, T_V128 = 0x7B,
       T_FUNCREF = 0x70, T_EXTERNREF = 0x6F, T_UNKNOWN = 0 };

/* ErrCode values (include/common/enum.inc:573-749) */
enum { E_OK = 0, E_TERMINATED = 0x01, E_COST_LIMIT = 0x03, E_FUNC_NOT_FOUND = 0x05, E_MALFORMED = 0x21,
       E_ILLEGAL_OPCODE = 0x37, E_TYPECHECK = 0x41, E_FUNCSIG = 0x83, E_DIV0 = 0x84,
       E_INTOVF = 0x85, E_CONV = 0x86, E_TABLE_OOB = 0x87, E_MEM_OOB = 0x88,
       E_UNREACHABLE = 0x89, E_UNINIT_ELEM = 0x8A, E_UNDEF_ELEM = 0x8B,
       E_INDIRECT_MISMATCH = 0x8C, E_HOST_FAILED = 0x8D, E_DATASEG = 0x63,
       E_ELEMSEG = 0x64, E_UNKNOWN_IMPORT = 0x62 };

#define REF_NULL UINT64_MAX        /* null reference in a slot */
#define PAGE 65536u
#define OM_MAX_XMEM 7              /* memories past the first (MultiMemories) */

typedef struct {
  uint16_t op;
  uint8_t is_last;
  uint8_t lane;
  uint32_t jump_end, jump_else;
  int32_t bt;                       /* blocktype: -64 empty, <0 valtype, >=0 type idx */
  uint32_t idx, idx2;               /* target / source index */
  uint32_t stack_offset;            /* local.* (formchecker.cpp:664-666) */
  uint32_t erase_begin, erase_end;  /* br / br_if Jump descriptor */
  int32_t pc_off;
  uint32_t lt_start, lt_n;          /* br_table label list (pool) */
  uint32_t mem_off;
  uint8_t mem, mem2;                /* memory index (MultiMemories; memory.copy: dst, src) */
  Val num;                          /* const immediate / v128 / shuffle mask */
} Instr;

typedef struct { uint32_t target, erase_begin, erase_end; int32_t pc_off; } Label;

typedef struct { uint32_t np, nr; uint8_t p[64], r[64]; } FType;

typedef struct {
  uint32_t type;
  uint32_t nlocals;                 /* declared locals (not params) */
  uint8_t *ltypes;                  /* params + locals */
  uint32_t start, len;              /* range into code[] */
  int imported;
  char imod[32], iname[32];         /* import names (imports only) */
} Func;

typedef struct { uint8_t reftype; uint32_t min, max; int has_max; } TableT;
typedef struct { uint8_t type, mut; uint32_t init_start, init_len; int imported; uint64_t lo, hi; } GlobalT;
typedef struct { char *name; uint8_t kind; uint32_t idx; } Export;
typedef struct {
  int mode;                          /* 0 active, 1 passive, 2 declarative */
  uint32_t table; uint32_t off_start, off_len; uint32_t n;
  uint32_t *items_start, *items_len; /* each item is a const expr range */
} Elem;
typedef struct { int mode; uint32_t off_start, off_len; uint8_t *bytes; uint32_t len; uint32_t mem; } Data;

struct OMod {
  uint32_t ntypes; FType *types;
  uint32_t nfuncs, nimported; Func *funcs;
  Instr *code; uint32_t ncode, capcode;
  Label *labels; uint32_t nlabels, caplabels;
  uint32_t ntables; TableT *tables;
  int has_mem; uint32_t mem_min, mem_max; int mem_has_max;
  /* memories 1..nxmem (the MultiMemories proposal): limits of memory k at [k - 1] */
  uint32_t nxmem; uint32_t xmin[OM_MAX_XMEM], xmax[OM_MAX_XMEM]; int xhas_max[OM_MAX_XMEM];
  uint32_t nglobals; GlobalT *globals;
  uint32_t nexports; Export *exports;
  int64_t start;
  uint32_t nelems; Elem *elems;
  uint32_t ndatas; Data *datas;
  uint32_t page_limit;
};

typedef struct { uint32_t size; uint64_t *refs; uint32_t max; int has_max; } TableI;

struct OInst {
  OMod *m;
  uint8_t *mem; uint32_t pages;
  /* memories 1..nxmem; sel = the memory now in mem/pages (xmem_exec swaps, 0 otherwise) */
  uint8_t *xmem[OM_MAX_XMEM]; uint32_t xpages[OM_MAX_XMEM]; uint32_t sel;
  Val *globals;
  TableI *tables;
  int *elem_dropped, *data_dropped;
  /* StackManager (stackmgr.h:25-148) */
  Val *vs; uint64_t vsp, vcap;
  struct Frame { int has_module; uint32_t from; uint32_t locals, arity; uint64_t vpos; } *fs;
  uint64_t fsp, fcap;
  uint64_t count;
  int terminated;                   /* the last invoke ended in Terminated (proc_exit) */
  /* gas (statistics.h:32,69-91): Statistics::CostSum belongs to the VM and is never reset
   * between executions, so it runs on from instantiation (constant expressions, start
   * function) across every invocation of this instance */
  int metered;
  uint64_t cost_limit, cost_sum;
  const uint64_t *cost_tab;         /* 65536 entries by OpCode; NULL = the unit table */
  uint64_t mem_bytes;               /* linear-memory bytes the last invoke accessed (not
                                       in the reference: the roofline's algorithmic bytes) */
  uint64_t mem_store_bytes;         /* ... of them written (stores, bulk destinations) */
  /* WASI subset (wasifunc.cpp): captured fd 1 / fd 2 bytes and the proc_exit code */
  uint8_t *wasi_out[2]; uint64_t wasi_len[2], wasi_cap[2];
  uint32_t wasi_exit;
  char **own_args; uint32_t own_nargs; int has_own_args;   /* this VM's own command line */
  /* WASI fd table (Environ::FdMap; wasi_fs.inc), the lane's generator and clock calls */
  struct WFd *wfd; uint32_t nwfd, capwfd; int wfd_init;
  uint64_t wrng, wclock; uint32_t wasi_lane;
};

/* ------------------------------------------------------------------ reader */
typedef struct { const uint8_t *p, *end; int err; } Rd;

static uint8_t rd_u8(Rd *r) {
  if (r->p >= r->end) { r->err = E_MALFORMED; return 0; }
  return *r->p++;
}
static uint64_t rd_uleb(Rd *r, int bits) {
  uint64_t v = 0; int sh = 0;
  for (;;) {
    uint8_t b = rd_u8(r);
    if (r->err) return 0;
    v |= (uint64_t)(b & 0x7F) << sh;
    sh += 7;
    if (!(b & 0x80)) break;
    if (sh >= bits + 7) { r->err = E_MALFORMED; return 0; }
  }
  return v;
}
static int64_t rd_sleb(Rd *r, int bits) {
  int64_t v = 0; int sh = 0; uint8_t b;
  do {
    b = rd_u8(r);
    if (r->err) return 0;
    v |= (int64_t)(b & 0x7F) << sh;
    sh += 7;
    if (sh >= bits + 7) { r->err = E_MALFORMED; return 0; }
  } while (b & 0x80);
  if (sh < 64 && (b & 0x40)) v |= -((int64_t)1 << sh);
  return v;
}
static uint32_t rd_u32(Rd *r) { return (uint32_t)rd_uleb(r, 32); }

/* ------------------------------------------------------------------ module growth */
static uint32_t push_instr(OMod *m) {
  if (m->ncode == m->capcode) {
    m->capcode = m->capcode ? m->capcode * 2 : 1024;
    m->code = realloc(m->code, sizeof(Instr) * m->capcode);
  }
  memset(&m->code[m->ncode], 0, sizeof(Instr));
  return m->ncode++;
}
static uint32_t push_label(OMod *m) {
  if (m->nlabels == m->caplabels) {
    m->caplabels = m->caplabels ? m->caplabels * 2 : 256;
    m->labels = realloc(m->labels, sizeof(Label) * m->caplabels);
  }
  memset(&m->labels[m->nlabels], 0, sizeof(Label));
  return m->nlabels++;
}

/* The MultiMemories proposal (configure.h:176-182: off by default); TEST INFRASTRUCTURE
 * knob mirroring WasmEdge_BatchConfigure::MultiMemories for modules loaded from now on. */
static int g_multi_memory;
void om_set_multi_memory(int on) { g_multi_memory = on != 0; }

/* a memory index immediate (instruction.cpp:374-389): a u32 with MultiMemories, else a
 * zero byte; past 255 (no module has that many memories) it is unknown anyway */
static uint8_t rd_memidx(Rd *r, int *bad) {
  if (!g_multi_memory) { if (rd_u8(r) != 0) *bad = 1; return 0; }
  uint32_t x = rd_u32(r);
  return x > 255 ? 255 : (uint8_t)x;
}
/* memarg (instruction.cpp:144-156): align, offset, then -- with MultiMemories and align
 * >= 64 -- the memory index */
static void rd_memarg(Rd *r, Instr *in) {
  uint32_t al = rd_u32(r);
  in->mem_off = rd_u32(r);
  if (g_multi_memory && al >= 64) { uint32_t x = rd_u32(r); in->mem = x > 255 ? 255 : (uint8_t)x; }
}

/* Immediates of one instruction (lib/loader/ast/instruction.cpp loadInstruction). */
static int load_immediates(OMod *m, Rd *r, uint32_t ii) {
  Instr *in = &m->code[ii];
  uint16_t op = in->op;
  switch (op) {
  case 0x02: case 0x03: case 0x04: {
    uint8_t b = *r->p;
    if (b == 0x40) { r->p++; in->bt = -64; }
    else if (b == T_I32 || b == T_I64 || b == T_F32 || b == T_F64 || b == T_V128 ||
             b == T_FUNCREF || b == T_EXTERNREF) { r->p++; in->bt = -(int32_t)b; }
    else in->bt = (int32_t)rd_sleb(r, 33);
    break;
  }
  case 0x0C: case 0x0D: in->idx = rd_u32(r); break;
  case 0x0E: {
    uint32_t n = rd_u32(r);
    in->lt_start = m->nlabels; in->lt_n = n + 1;
    for (uint32_t k = 0; k <= n; k++) {
      uint32_t t = rd_u32(r);
      uint32_t li = push_label(m);
      m->labels[li].target = t;
      in = &m->code[ii];
    }
    break;
  }
  case 0x10: case 0x12: case 0xD2: in->idx = rd_u32(r); break;
  case 0x11: case 0x13: in->idx = rd_u32(r); in->idx2 = rd_u32(r); break;
  case 0x1C: { uint32_t n = rd_u32(r); for (uint32_t k = 0; k < n; k++) in->idx = rd_u8(r);
               if (n != 1) return E_TYPECHECK; break; }
  case 0x20: case 0x21: case 0x22: case 0x23: case 0x24: case 0x25: case 0x26:
    in->idx = rd_u32(r); break;
  case 0x3F: case 0x40: { int bad = 0; in->mem = rd_memidx(r, &bad); if (bad) return E_MALFORMED; break; }
  case 0x41: in->num.lo = (uint32_t)(int32_t)rd_sleb(r, 32); break;
  case 0x42: in->num.lo = (uint64_t)rd_sleb(r, 64); break;
  case 0x43: { uint32_t v = 0; for (int k = 0; k < 4; k++) v |= (uint32_t)rd_u8(r) << (8 * k);
               in->num.lo = v; break; }
  case 0x44: { uint64_t v = 0; for (int k = 0; k < 8; k++) v |= (uint64_t)rd_u8(r) << (8 * k);
               in->num.lo = v; break; }
  case 0xD0: in->idx = rd_u8(r); break;
  case 0xFC08: {
    int bad = 0;
    in->idx = rd_u32(r);
    in->mem = rd_memidx(r, &bad);
    if (bad) return E_MALFORMED;
    break;
  }
  case 0xFC09: in->idx = rd_u32(r); break;
  case 0xFC0A: {
    int bad = 0;
    in->mem = rd_memidx(r, &bad);
    in->mem2 = rd_memidx(r, &bad);
    if (bad) return E_MALFORMED;
    break;
  }
  case 0xFC0B: { int bad = 0; in->mem = rd_memidx(r, &bad); if (bad) return E_MALFORMED; break; }
  case 0xFC0C: in->idx2 = rd_u32(r); in->idx = rd_u32(r); break;   /* elem, table */
  case 0xFC0D: in->idx = rd_u32(r); break;
  case 0xFC0E: in->idx = rd_u32(r); in->idx2 = rd_u32(r); break;   /* dst, src */
  case 0xFC0F: case 0xFC10: case 0xFC11: in->idx = rd_u32(r); break;
  case 0xFD0C: case 0xFD0D: {
    uint64_t lo = 0, hi = 0;
    for (int k = 0; k < 8; k++) lo |= (uint64_t)rd_u8(r) << (8 * k);
    for (int k = 0; k < 8; k++) hi |= (uint64_t)rd_u8(r) << (8 * k);
    in->num.lo = lo; in->num.hi = hi;
    break;
  }
  default:
    if ((op >= 0x28 && op <= 0x3E) || (op >= 0xFD00 && op <= 0xFD0B) || op == 0xFD5C ||
        op == 0xFD5D) {
      rd_memarg(r, in);
    } else if (op >= 0xFD54 && op <= 0xFD5B) {
      rd_memarg(r, in); in->lane = rd_u8(r);
    } else if (op >= 0xFD15 && op <= 0xFD22) {
      in->lane = rd_u8(r);
    }
  }
  return r->err;
}

/* The TailCall proposal (configure.h:176-182: off by default); TEST INFRASTRUCTURE knob
 * mirroring WasmEdge_BatchConfigure::TailCall for modules loaded from now on. */
static int g_tail_call;
void om_set_tail_call(int on) { g_tail_call = on != 0; }

/* lib/loader/ast/instruction.cpp:35-116 -- decode one expression with block stack. */
static int load_instr_seq(OMod *m, Rd *r, uint32_t *start, uint32_t *len) {
  uint32_t bstack[1024], bsp = 0;
  uint32_t first = m->ncode;
  for (;;) {
    uint16_t op = rd_u8(r);
    if (op == 0xFC || op == 0xFD) {
      uint32_t sub = rd_u32(r);
      if (sub > 0xFF) return E_ILLEGAL_OPCODE;
      op = (uint16_t)(op << 8 | sub);
    }
    if (r->err) return r->err;
    /* instruction.cpp:903-907: return_call(_indirect) need the TailCall proposal */
    if ((op == 0x12 || op == 0x13) && !g_tail_call) return E_ILLEGAL_OPCODE;
    uint32_t ii = push_instr(m);
    m->code[ii].op = op;
    int reach_end = 0;
    if (op == 0x02 || op == 0x03 || op == 0x04) {
      if (bsp == 1024) return E_MALFORMED;
      bstack[bsp++] = ii;
    } else if (op == 0x05) {
      if (!bsp || m->code[bstack[bsp - 1]].op != 0x04) return E_ILLEGAL_OPCODE;
      uint32_t pos = bstack[bsp - 1];
      if (m->code[pos].jump_else) return E_ILLEGAL_OPCODE;
      m->code[pos].jump_else = ii - pos;
    } else if (op == 0x0B) {
      if (bsp) {
        uint32_t pos = bstack[--bsp];
        m->code[pos].jump_end = ii - pos;
        if (m->code[pos].op == 0x04) {
          if (m->code[pos].jump_else == 0) m->code[pos].jump_else = ii - pos;
          else {
            uint32_t ep = pos + m->code[pos].jump_else;
            m->code[ep].jump_end = ii - ep;
          }
        }
      } else reach_end = 1;
    }
    int e = load_immediates(m, r, ii);
    if (e) return e;
    if (op == 0x0B) m->code[ii].is_last = (uint8_t)reach_end;
    if (reach_end) break;
  }
  *start = first;
  *len = m->ncode - first;
  return 0;
}

/* ------------------------------------------------------------------ validation
 * FormChecker restated: operand type stack + control stack; writes the jump
 * descriptors and StackOffsets into the Instr records. */
typedef struct {
  uint8_t start_t[64], end_t[64]; uint32_t ns, ne;
  uint32_t jump;     /* instruction index the label jumps to */
  uint64_t height;
  uint16_t code;
  int unreachable;
} Ctrl;

typedef struct {
  OMod *m;
  uint8_t *vals; uint64_t nv, capv;
  Ctrl *ctrl; uint32_t nc, capc;
  uint8_t *locals; uint32_t nlocals;
  uint8_t returns[64]; uint32_t nret;
  int err;
} Chk;

static void ck_push(Chk *c, uint8_t t) {
  if (c->nv == c->capv) { c->capv = c->capv ? 2 * c->capv : 256; c->vals = realloc(c->vals, c->capv); }
  c->vals[c->nv++] = t;
}
static uint8_t ck_pop(Chk *c) {
  Ctrl *f = &c->ctrl[c->nc - 1];
  if (c->nv == f->height) {
    if (f->unreachable) return T_UNKNOWN;
    c->err = E_TYPECHECK; return T_UNKNOWN;
  }
  return c->vals[--c->nv];
}
static uint8_t ck_pop_t(Chk *c, uint8_t want) {
  uint8_t t = ck_pop(c);
  if (t != T_UNKNOWN && want != T_UNKNOWN && t != want) c->err = E_TYPECHECK;
  return t == T_UNKNOWN ? want : t;
}
static void ck_pops(Chk *c, const uint8_t *ts, uint32_t n) {
  for (uint32_t k = n; k > 0; k--) ck_pop_t(c, ts[k - 1]);
}
static void ck_pushs(Chk *c, const uint8_t *ts, uint32_t n) {
  for (uint32_t k = 0; k < n; k++) ck_push(c, ts[k]);
}
static void ck_push_ctrl(Chk *c, const uint8_t *in, uint32_t ni, const uint8_t *out,
                         uint32_t no, uint32_t jump, uint16_t code) {
  if (c->nc == c->capc) { c->capc = c->capc ? 2 * c->capc : 64; c->ctrl = realloc(c->ctrl, sizeof(Ctrl) * c->capc); }
  Ctrl *f = &c->ctrl[c->nc++];
  memcpy(f->start_t, in, ni); f->ns = ni;
  memcpy(f->end_t, out, no); f->ne = no;
  f->jump = jump; f->height = c->nv; f->code = code; f->unreachable = 0;
  ck_pushs(c, in, ni);
}
static void ck_unreachable(Chk *c) {       /* formchecker.cpp:1413-1421 */
  Ctrl *f = &c->ctrl[c->nc - 1];
  c->nv = f->height;
  f->unreachable = 1;
}
static int ck_pop_ctrl(Chk *c, Ctrl *out) {
  if (!c->nc) return E_TYPECHECK;
  Ctrl *f = &c->ctrl[c->nc - 1];
  ck_pops(c, f->end_t, f->ne);
  if (c->nv != f->height) return E_TYPECHECK;
  *out = *f;
  c->nc--;
  return c->err;
}
static void label_types(const Ctrl *f, const uint8_t **t, uint32_t *n) {
  if (f->code == 0x03) { *t = f->start_t; *n = f->ns; } else { *t = f->end_t; *n = f->ne; }
}
static int block_type(OMod *m, int32_t bt, const uint8_t **in, uint32_t *ni,
                      const uint8_t **out, uint32_t *no, uint8_t *buf) {
  if (bt == -64) { *ni = *no = 0; *in = *out = buf; return 0; }
  if (bt < 0) { buf[0] = (uint8_t)(-bt); *in = buf; *ni = 0; *out = buf; *no = 1; return 0; }
  if ((uint32_t)bt >= m->ntypes) return E_TYPECHECK;
  *in = m->types[bt].p; *ni = m->types[bt].np; *out = m->types[bt].r; *no = m->types[bt].nr;
  return 0;
}

/* Stack signature of the plain (non-control, non-variable) opcodes.
 * Encoded "pops:pushes" with i=i32 l=i64 f=f32 d=f64 v=v128. */
static const char *simple_sig(uint16_t op) {
  if (op >= 0x45 && op <= 0xC4) {
    if (op == 0x45) return "i:i";
    if (op <= 0x4F) return "ii:i";
    if (op == 0x50) return "l:i";
    if (op <= 0x5A) return "ll:i";
    if (op <= 0x60) return "ff:i";
    if (op <= 0x66) return "dd:i";
    if (op <= 0x69) return "i:i";
    if (op <= 0x78) return "ii:i";
    if (op <= 0x7B) return "l:l";
    if (op <= 0x8A) return "ll:l";
    if (op <= 0x91) return "f:f";
    if (op <= 0x98) return "ff:f";
    if (op <= 0x9F) return "d:d";
    if (op <= 0xA6) return "dd:d";
    switch (op) {
    case 0xA7: return "l:i"; case 0xA8: case 0xA9: return "f:i"; case 0xAA: case 0xAB: return "d:i";
    case 0xAC: case 0xAD: return "i:l"; case 0xAE: case 0xAF: return "f:l";
    case 0xB0: case 0xB1: return "d:l"; case 0xB2: case 0xB3: return "i:f";
    case 0xB4: case 0xB5: return "l:f"; case 0xB6: return "d:f"; case 0xB7: case 0xB8: return "i:d";
    case 0xB9: case 0xBA: return "l:d"; case 0xBB: return "f:d"; case 0xBC: return "f:i";
    case 0xBD: return "d:l"; case 0xBE: return "i:f"; case 0xBF: return "l:d";
    case 0xC0: case 0xC1: return "i:i"; default: return "l:l";
    }
  }
  if (op >= 0xFC00 && op <= 0xFC07) {
    static const char *s[8] = {"f:i", "f:i", "d:i", "d:i", "f:l", "f:l", "d:l", "d:l"};
    return s[op - 0xFC00];
  }
  if (op >= 0x28 && op <= 0x35) {
    static const char *s[] = {"i:i", "i:l", "i:f", "i:d", "i:i", "i:i", "i:i", "i:i",
                              "i:l", "i:l", "i:l", "i:l", "i:l", "i:l"};
    return s[op - 0x28];
  }
  if (op >= 0x36 && op <= 0x3E) {
    static const char *s[] = {"ii:", "il:", "if:", "id:", "ii:", "ii:", "il:", "il:", "il:"};
    return s[op - 0x36];
  }
  if (op >= 0xFD00) {
    uint8_t s = (uint8_t)op;
    if (s <= 0x0A || s == 0x5C || s == 0x5D) return "i:v";
    if (s == 0x0B) return "iv:";
    if (s >= 0x54 && s <= 0x57) return "iv:v";
    if (s >= 0x58 && s <= 0x5B) return "iv:";
    if (s == 0x0C) return ":v";
    if (s == 0x0D || s == 0x0E) return "vv:v";
    switch (s) {
    case 0x0F: case 0x10: case 0x11: return "i:v";
    case 0x12: return "l:v"; case 0x13: return "f:v"; case 0x14: return "d:v";
    case 0x15: case 0x16: case 0x18: case 0x19: case 0x1B: return "v:i";
    case 0x17: case 0x1A: case 0x1C: return "vi:v";
    case 0x1D: return "v:l"; case 0x1E: return "vl:v";
    case 0x1F: return "v:f"; case 0x20: return "vf:v";
    case 0x21: return "v:d"; case 0x22: return "vd:v";
    case 0x4D: return "v:v"; case 0x52: return "vvv:v"; case 0x53: return "v:i";
    case 0x63: case 0x64: case 0x83: case 0x84: case 0xA3: case 0xA4: case 0xC3: case 0xC4:
      return "v:i";
    case 0x6B: case 0x6C: case 0x6D: case 0x8B: case 0x8C: case 0x8D: case 0xAB: case 0xAC:
    case 0xAD: case 0xCB: case 0xCC: case 0xCD:
      return "vi:v";
    case 0x5E: case 0x5F: case 0x60: case 0x61: case 0x62: case 0x67: case 0x68: case 0x69:
    case 0x6A: case 0x74: case 0x75: case 0x7A: case 0x7C: case 0x7D: case 0x7E: case 0x7F:
    case 0x80: case 0x81: case 0x87: case 0x88: case 0x89: case 0x8A: case 0x94: case 0xA0:
    case 0xA1: case 0xA7: case 0xA8: case 0xA9: case 0xAA: case 0xC0: case 0xC1: case 0xC7:
    case 0xC8: case 0xC9: case 0xCA: case 0xE0: case 0xE1: case 0xE3: case 0xEC: case 0xED:
    case 0xEF: case 0xF8: case 0xF9: case 0xFA: case 0xFB: case 0xFC: case 0xFD: case 0xFE:
    case 0xFF:
      return "v:v";
    default: return "vv:v";
    }
  }
  return NULL;
}

static uint8_t sigc(char ch) {
  switch (ch) { case 'i': return T_I32; case 'l': return T_I64; case 'f': return T_F32;
                case 'd': return T_F64; default: return T_V128; }
}

/* a memory index of an instruction: unknown memory (InvalidMemoryIdx, formchecker.cpp:
 * 245-252) -- TypeCheckFailed without MultiMemories, as for a module without memory */
static int mem_idx_err(const OMod *m, uint32_t k) {
  const uint32_t nm = (m->has_mem ? 1u : 0u) + m->nxmem;
  if (k < nm) return 0;
  return g_multi_memory && nm ? 0x47 : E_TYPECHECK;
}

static int check_func(OMod *m, uint32_t fi) {
  Func *F = &m->funcs[fi];
  FType *ft = &m->types[F->type];
  Chk c; memset(&c, 0, sizeof c);
  c.m = m; c.locals = F->ltypes; c.nlocals = ft->np + F->nlocals;
  memcpy(c.returns, ft->r, ft->nr); c.nret = ft->nr;
  /* formchecker.cpp:188-191: function label jumps to the last instruction */
  ck_push_ctrl(&c, NULL, 0, ft->r, ft->nr, F->start + F->len - 1, 0x02);
  for (uint32_t k = 0; k < F->len && !c.err; k++) {
    uint32_t ii = F->start + k;
    Instr *in = &m->code[ii];
    uint16_t op = in->op;
    const uint8_t *t1, *t2; uint32_t n1, n2; uint8_t buf[1];
    switch (op) {
    case 0x00: ck_unreachable(&c); break;
    case 0x01: break;
    case 0x04: ck_pop_t(&c, T_I32); /* fallthrough */
    case 0x02: case 0x03: {
      if ((c.err = block_type(m, in->bt, &t1, &n1, &t2, &n2, buf))) break;
      uint8_t bt1[64], bt2[64];
      memcpy(bt1, t1, n1); memcpy(bt2, t2, n2);
      ck_pops(&c, bt1, n1);
      uint32_t jump = (op == 0x03) ? ii : ii + in->jump_end;
      ck_push_ctrl(&c, bt1, n1, bt2, n2, jump, op);
      if (op == 0x04 && in->jump_else == in->jump_end) {
        if (n1 != n2 || memcmp(bt1, bt2, n1)) c.err = E_TYPECHECK;
      }
      break;
    }
    case 0x05: {
      Ctrl f;
      if ((c.err = ck_pop_ctrl(&c, &f))) break;
      ck_push_ctrl(&c, f.start_t, f.ns, f.end_t, f.ne, f.jump, op);
      break;
    }
    case 0x0B: {
      Ctrl f;
      if ((c.err = ck_pop_ctrl(&c, &f))) break;
      ck_pushs(&c, f.end_t, f.ne);
      break;
    }
    case 0x0C: case 0x0D: {
      if (in->idx >= c.nc) { c.err = E_TYPECHECK; break; }
      Ctrl *f = &c.ctrl[c.nc - 1 - in->idx];
      if (op == 0x0D) ck_pop_t(&c, T_I32);
      const uint8_t *lt; uint32_t ln; label_types(f, &lt, &ln);
      uint8_t tmp[64]; memcpy(tmp, lt, ln);
      ck_pops(&c, tmp, ln);
      uint32_t remain = (uint32_t)(c.nv - f->height);
      in->erase_begin = remain + ln; in->erase_end = ln;
      in->pc_off = (int32_t)f->jump - (int32_t)ii;
      if (op == 0x0C) ck_unreachable(&c); else ck_pushs(&c, tmp, ln);
      break;
    }
    case 0x0E: {
      ck_pop_t(&c, T_I32);
      uint32_t n = in->lt_n;
      Label *L = &m->labels[in->lt_start];
      for (uint32_t k2 = 0; k2 < n; k2++) {
        if (L[k2].target >= c.nc) { c.err = E_TYPECHECK; break; }
      }
      if (c.err) break;
      Ctrl *fm = &c.ctrl[c.nc - 1 - L[n - 1].target];
      const uint8_t *mt; uint32_t mn; label_types(fm, &mt, &mn);
      for (uint32_t k2 = 0; k2 + 1 < n; k2++) {
        Ctrl *fn = &c.ctrl[c.nc - 1 - L[k2].target];
        const uint8_t *nt; uint32_t nn; label_types(fn, &nt, &nn);
        if (nn != mn) { c.err = E_TYPECHECK; break; }
        uint8_t tb[64];
        for (uint32_t q = nn; q > 0; q--) {
          uint8_t got = ck_pop_t(&c, nt[q - 1]);
          tb[q - 1] = c.ctrl[c.nc - 1].unreachable ? T_UNKNOWN : got;
        }
        uint32_t remain = (uint32_t)(c.nv - fn->height);
        L[k2].erase_begin = remain + nn; L[k2].erase_end = nn;
        L[k2].pc_off = (int32_t)fn->jump - (int32_t)ii;
        ck_pushs(&c, tb, nn);
      }
      uint8_t tmp[64]; memcpy(tmp, mt, mn);
      ck_pops(&c, tmp, mn);
      uint32_t remain = (uint32_t)(c.nv - fm->height);
      L[n - 1].erase_begin = remain + mn; L[n - 1].erase_end = mn;
      L[n - 1].pc_off = (int32_t)fm->jump - (int32_t)ii;
      ck_unreachable(&c);
      break;
    }
    case 0x0F: ck_pops(&c, c.returns, c.nret); ck_unreachable(&c); break;
    case 0x10: case 0x12: {
      if (in->idx >= m->nfuncs) { c.err = E_TYPECHECK; break; }
      FType *t = &m->types[m->funcs[in->idx].type];
      /* formchecker.cpp:526-530: a tail call's callee returns what the caller returns */
      if (op == 0x12 && (t->nr != c.nret || memcmp(t->r, c.returns, t->nr))) { c.err = E_TYPECHECK; break; }
      ck_pops(&c, t->p, t->np);
      if (op == 0x12) { ck_unreachable(&c); break; }
      ck_pushs(&c, t->r, t->nr);
      break;
    }
    case 0x11: case 0x13: {
      if (in->idx >= m->ntypes || in->idx2 >= m->ntables) { c.err = E_TYPECHECK; break; }
      ck_pop_t(&c, T_I32);
      FType *t = &m->types[in->idx];
      if (op == 0x13 && (t->nr != c.nret || memcmp(t->r, c.returns, t->nr))) { c.err = E_TYPECHECK; break; }
      ck_pops(&c, t->p, t->np);
      if (op == 0x13) { ck_unreachable(&c); break; }
      ck_pushs(&c, t->r, t->nr);
      break;
    }
    case 0xD0: ck_push(&c, (uint8_t)in->idx); break;
    case 0xD1: { uint8_t t = ck_pop(&c); if (t != T_UNKNOWN && t != T_FUNCREF && t != T_EXTERNREF) c.err = E_TYPECHECK; ck_push(&c, T_I32); break; }
    case 0xD2: ck_push(&c, T_FUNCREF); break;
    case 0x1A: ck_pop(&c); break;
    case 0x1B: {
      ck_pop_t(&c, T_I32);
      uint8_t a = ck_pop(&c), b = ck_pop(&c);
      if (a != T_UNKNOWN && b != T_UNKNOWN && a != b) c.err = E_TYPECHECK;
      ck_push(&c, a == T_UNKNOWN ? b : a);
      break;
    }
    case 0x1C: {
      uint8_t t = (uint8_t)in->idx;
      ck_pop_t(&c, T_I32); ck_pop_t(&c, t); ck_pop_t(&c, t); ck_push(&c, t);
      break;
    }
    case 0x20: case 0x21: case 0x22: {
      if (in->idx >= c.nlocals) { c.err = E_TYPECHECK; break; }
      uint8_t t = c.locals[in->idx];
      /* formchecker.cpp:664-666 */
      in->stack_offset = (uint32_t)((c.nv - c.ctrl[0].height) + (c.nlocals - in->idx));
      if (op == 0x20) ck_push(&c, t);
      else if (op == 0x21) ck_pop_t(&c, t);
      else { ck_pop_t(&c, t); ck_push(&c, t); }
      break;
    }
    case 0x23: case 0x24: {
      if (in->idx >= m->nglobals) { c.err = E_TYPECHECK; break; }
      uint8_t t = m->globals[in->idx].type;
      if (op == 0x23) ck_push(&c, t);
      else { if (!m->globals[in->idx].mut) c.err = E_TYPECHECK; ck_pop_t(&c, t); }
      break;
    }
    case 0x25: case 0x26: {
      if (in->idx >= m->ntables) { c.err = E_TYPECHECK; break; }
      uint8_t t = m->tables[in->idx].reftype;
      if (op == 0x25) { ck_pop_t(&c, T_I32); ck_push(&c, t); }
      else { ck_pop_t(&c, t); ck_pop_t(&c, T_I32); }
      break;
    }
    case 0x3F: if ((c.err = mem_idx_err(m, in->mem))) break; ck_push(&c, T_I32); break;
    case 0x40: if ((c.err = mem_idx_err(m, in->mem))) break; ck_pop_t(&c, T_I32); ck_push(&c, T_I32); break;
    case 0x41: ck_push(&c, T_I32); break;
    case 0x42: ck_push(&c, T_I64); break;
    case 0x43: ck_push(&c, T_F32); break;
    case 0x44: ck_push(&c, T_F64); break;
    case 0xFC08: if ((c.err = mem_idx_err(m, in->mem))) break;   /* (formchecker.cpp:812-824) */
      if (in->idx >= m->ndatas) c.err = g_multi_memory ? 0x4A : E_TYPECHECK;
      ck_pop_t(&c, T_I32); ck_pop_t(&c, T_I32); ck_pop_t(&c, T_I32); break;
    case 0xFC09: if (in->idx >= m->ndatas) c.err = E_TYPECHECK; break;
    case 0xFC0A: case 0xFC0B:   /* copy: the source memory first (formchecker.cpp:826-834) */
      if (op == 0xFC0A && (c.err = mem_idx_err(m, in->mem2))) break;
      if ((c.err = mem_idx_err(m, in->mem))) break;
      ck_pop_t(&c, T_I32); ck_pop_t(&c, T_I32); ck_pop_t(&c, T_I32); break;
    case 0xFC0C: if (in->idx >= m->ntables || in->idx2 >= m->nelems) c.err = E_TYPECHECK;
      ck_pop_t(&c, T_I32); ck_pop_t(&c, T_I32); ck_pop_t(&c, T_I32); break;
    case 0xFC0D: if (in->idx >= m->nelems) c.err = E_TYPECHECK; break;
    case 0xFC0E: if (in->idx >= m->ntables || in->idx2 >= m->ntables) c.err = E_TYPECHECK;
      ck_pop_t(&c, T_I32); ck_pop_t(&c, T_I32); ck_pop_t(&c, T_I32); break;
    case 0xFC0F: if (in->idx >= m->ntables) { c.err = E_TYPECHECK; break; }
      ck_pop_t(&c, T_I32); ck_pop_t(&c, m->tables[in->idx].reftype); ck_push(&c, T_I32); break;
    case 0xFC10: if (in->idx >= m->ntables) c.err = E_TYPECHECK; ck_push(&c, T_I32); break;
    case 0xFC11: if (in->idx >= m->ntables) { c.err = E_TYPECHECK; break; }
      ck_pop_t(&c, T_I32); ck_pop_t(&c, m->tables[in->idx].reftype); ck_pop_t(&c, T_I32); break;
    default: {
      const char *s = simple_sig(op);
      if (!s) { c.err = E_ILLEGAL_OPCODE; break; }
      if ((op >= 0x28 && op <= 0x3E) || (op >= 0xFD00 && op <= 0xFD0B) ||
          (op >= 0xFD54 && op <= 0xFD5D)) {
        if ((c.err = mem_idx_err(m, in->mem))) break;
      }
      const char *colon = strchr(s, ':');
      int np = (int)(colon - s);
      for (int q = np - 1; q >= 0; q--) ck_pop_t(&c, sigc(s[q]));
      for (const char *q = colon + 1; *q; q++) ck_push(&c, sigc(*q));
    }
    }
  }
  int err = c.err;
  if (!err && c.nc != 0) err = E_TYPECHECK;
  free(c.vals); free(c.ctrl);
  return err;
}

/* ------------------------------------------------------------------ module loading */
static int load_const_expr(OMod *m, Rd *r, uint32_t *start, uint32_t *len) {
  return load_instr_seq(m, r, start, len);
}

static int load_limits(Rd *r, uint32_t *mn, uint32_t *mx, int *has) {
  uint8_t f = rd_u8(r);
  *mn = rd_u32(r);
  *has = f & 1;
  *mx = *has ? rd_u32(r) : 0;
  return r->err;
}

/* TEST INFRASTRUCTURE: the tables / memories / globals the batched path's embedder
 * provides (WasmEdge_BatchCreateWithImports), for modules importing them. Matching
 * follows instantiate/import.cpp:35-42 (isLimitMatched) and :137-190. */
typedef struct { char mod[32], name[32]; uint8_t kind, type, mut; uint32_t min, max; int has_max;
                 uint64_t lo, hi; } ProvidedImport;
static ProvidedImport g_provided[64];
static int g_nprovided;
void om_clear_imports(void) { g_nprovided = 0; }
void om_add_import(const char *mod, const char *name, uint32_t kind, uint32_t type, uint32_t mut,
                   uint32_t min, uint32_t max, int has_max, uint64_t lo, uint64_t hi) {
  if (g_nprovided >= 64) return;
  ProvidedImport *p = &g_provided[g_nprovided++];
  memset(p, 0, sizeof *p);
  strncpy(p->mod, mod, 31); strncpy(p->name, name, 31);
  p->kind = (uint8_t)kind; p->type = (uint8_t)type; p->mut = (uint8_t)mut;
  p->min = min; p->max = max; p->has_max = has_max; p->lo = lo; p->hi = hi;
}
static int limits_ok(const ProvidedImport *p, uint32_t min, int has_max, uint32_t max) {
  if (p->min < min || (!p->has_max && has_max)) return 0;
  if (p->has_max && has_max && p->max > max) return 0;
  return 1;
}
static int import_entity(OMod *m, Rd *s, uint8_t kind, const char *mod, const char *name) {
  uint8_t ty = 0, mut = 0;
  uint32_t mn = 0, mx = 0; int hm = 0;
  if (kind == 1) { ty = rd_u8(s); load_limits(s, &mn, &mx, &hm); }
  else if (kind == 2) load_limits(s, &mn, &mx, &hm);
  else if (kind == 3) { ty = rd_u8(s); mut = rd_u8(s); }
  else return E_MALFORMED;
  const ProvidedImport *p = NULL;
  for (int k = 0; k < g_nprovided; k++)
    if (g_provided[k].kind == kind && !strcmp(g_provided[k].mod, mod) && !strcmp(g_provided[k].name, name)) {
      p = &g_provided[k];
      break;
    }
  if (!p) return E_UNKNOWN_IMPORT;
  if (kind == 1) {
    if (p->type != ty || !limits_ok(p, mn, hm, mx)) return 0x61;
    m->tables = realloc(m->tables, sizeof(TableT) * (m->ntables + 2));
    TableT *t = &m->tables[m->ntables++];
    t->reftype = p->type; t->min = p->min; t->max = p->max; t->has_max = p->has_max;
  } else if (kind == 2) {
    if (m->has_mem && !g_multi_memory) return 0x51;   /* (validator.cpp:107-113) */
    if (!limits_ok(p, mn, hm, mx)) return 0x61;
    if (m->has_mem) {
      if (m->nxmem >= OM_MAX_XMEM) return 0x51;
      m->xmin[m->nxmem] = p->min; m->xmax[m->nxmem] = p->max; m->xhas_max[m->nxmem] = p->has_max;
      m->nxmem++;
    } else {
      m->has_mem = 1; m->mem_min = p->min; m->mem_max = p->max; m->mem_has_max = p->has_max;
    }
  } else {
    if (p->type != ty || p->mut != mut) return 0x61;
    m->globals = realloc(m->globals, sizeof(GlobalT) * (m->nglobals + 2));
    GlobalT *g = &m->globals[m->nglobals++];
    memset(g, 0, sizeof *g);
    g->type = ty; g->mut = mut; g->imported = 1; g->lo = p->lo; g->hi = p->hi;
  }
  return 0;
}

OMod *om_load(const uint8_t *wasm, uint32_t len, uint32_t page_limit, int *err) {
  OMod *m = calloc(1, sizeof(OMod));
  m->page_limit = page_limit ? page_limit : 65536;
  m->start = -1;
  Rd r = {wasm, wasm + len, 0};
  *err = 0;
  if (len < 8 || memcmp(wasm, "\0asm\1\0\0\0", 8)) { *err = E_MALFORMED; om_free(m); return NULL; }
  r.p += 8;
  uint32_t *func_types = NULL, nfunc_decl = 0;
  while (r.p < r.end && !*err) {
    uint8_t sid = rd_u8(&r);
    uint32_t slen = rd_u32(&r);
    const uint8_t *send = r.p + slen;
    if (send > r.end) { *err = E_MALFORMED; break; }
    Rd s = {r.p, send, 0};
    switch (sid) {
    case 0: break;
    case 1: {
      m->ntypes = rd_u32(&s);
      m->types = calloc(m->ntypes ? m->ntypes : 1, sizeof(FType));
      for (uint32_t k = 0; k < m->ntypes; k++) {
        if (rd_u8(&s) != 0x60) { *err = E_MALFORMED; break; }
        FType *t = &m->types[k];
        t->np = rd_u32(&s); if (t->np > 64) { *err = E_MALFORMED; break; }
        for (uint32_t q = 0; q < t->np; q++) t->p[q] = rd_u8(&s);
        t->nr = rd_u32(&s); if (t->nr > 64) { *err = E_MALFORMED; break; }
        for (uint32_t q = 0; q < t->nr; q++) t->r[q] = rd_u8(&s);
      }
      break;
    }
    case 2: {
      uint32_t n = rd_u32(&s);
      for (uint32_t k = 0; k < n; k++) {
        char nm[2][32] = {{0}};
        for (int q = 0; q < 2; q++) {
          uint32_t l = rd_u32(&s);
          if (s.p + l > s.end) { *err = E_MALFORMED; break; }
          memcpy(nm[q], s.p, l < 31 ? l : 31);
          s.p += l;
        }
        uint8_t kind = rd_u8(&s);
        if (kind != 0) {            /* table / memory / global: instantiate/import.cpp */
          if ((*err = import_entity(m, &s, kind, nm[0], nm[1]))) break;
          continue;
        }
        uint32_t ti = rd_u32(&s);
        m->funcs = realloc(m->funcs, sizeof(Func) * (m->nfuncs + 1));
        memset(&m->funcs[m->nfuncs], 0, sizeof(Func));
        m->funcs[m->nfuncs].type = ti;
        memcpy(m->funcs[m->nfuncs].imod, nm[0], 32);
        memcpy(m->funcs[m->nfuncs].iname, nm[1], 32);
        m->funcs[m->nfuncs].imported = 1;
        m->nfuncs++; m->nimported++;
      }
      break;
    }
    case 3: {
      nfunc_decl = rd_u32(&s);
      func_types = calloc(nfunc_decl + 1, sizeof(uint32_t));
      for (uint32_t k = 0; k < nfunc_decl; k++) func_types[k] = rd_u32(&s);
      break;
    }
    case 4: {                       /* after any imported tables */
      uint32_t n = rd_u32(&s), t0 = m->ntables;
      m->tables = realloc(m->tables, sizeof(TableT) * (t0 + n + 1));
      for (uint32_t k = 0; k < n; k++) {
        memset(&m->tables[t0 + k], 0, sizeof(TableT));
        m->tables[t0 + k].reftype = rd_u8(&s);
        load_limits(&s, &m->tables[t0 + k].min, &m->tables[t0 + k].max, &m->tables[t0 + k].has_max);
      }
      m->ntables = t0 + n;
      break;
    }
    case 5: {
      uint32_t n = rd_u32(&s);
      if (!g_multi_memory && (n > 1 || (n && m->has_mem))) { *err = 0x51; break; }
      for (uint32_t k = 0; k < n && !*err; k++) {
        if (!m->has_mem) {
          m->has_mem = 1;
          *err = load_limits(&s, &m->mem_min, &m->mem_max, &m->mem_has_max);
        } else if (m->nxmem >= OM_MAX_XMEM) {
          *err = 0x51;
        } else {
          *err = load_limits(&s, &m->xmin[m->nxmem], &m->xmax[m->nxmem], &m->xhas_max[m->nxmem]);
          m->nxmem++;
        }
      }
      break;
    }
    case 6: {                       /* after any imported globals */
      uint32_t n = rd_u32(&s), g0 = m->nglobals;
      m->globals = realloc(m->globals, sizeof(GlobalT) * (g0 + n + 1));
      for (uint32_t k = 0; k < n && !*err; k++) {
        GlobalT *g = &m->globals[g0 + k];
        memset(g, 0, sizeof(GlobalT));
        g->type = rd_u8(&s);
        g->mut = rd_u8(&s);
        *err = load_const_expr(m, &s, &g->init_start, &g->init_len);
      }
      m->nglobals = g0 + n;
      break;
    }
    case 7: {
      m->nexports = rd_u32(&s);
      m->exports = calloc(m->nexports + 1, sizeof(Export));
      for (uint32_t k = 0; k < m->nexports; k++) {
        uint32_t l = rd_u32(&s);
        m->exports[k].name = calloc(l + 1, 1);
        memcpy(m->exports[k].name, s.p, l); s.p += l;
        m->exports[k].kind = rd_u8(&s);
        m->exports[k].idx = rd_u32(&s);
      }
      break;
    }
    case 8: m->start = rd_u32(&s); break;
    case 9: {
      m->nelems = rd_u32(&s);
      m->elems = calloc(m->nelems + 1, sizeof(Elem));
      for (uint32_t k = 0; k < m->nelems && !*err; k++) {
        Elem *e = &m->elems[k];
        uint32_t flags = rd_u32(&s);
        e->mode = (flags & 1) ? ((flags & 2) ? 2 : 1) : 0;
        if (!(flags & 1)) {
          if (flags & 2) e->table = rd_u32(&s);
          *err = load_const_expr(m, &s, &e->off_start, &e->off_len);
        }
        if (flags & 3) rd_u8(&s);           /* elemkind or reftype */
        e->n = rd_u32(&s);
        e->items_start = calloc(e->n + 1, 4); e->items_len = calloc(e->n + 1, 4);
        for (uint32_t q = 0; q < e->n && !*err; q++) {
          if (flags & 4) {
            *err = load_const_expr(m, &s, &e->items_start[q], &e->items_len[q]);
          } else {
            /* store as a synthetic ref.func const expr */
            uint32_t a = push_instr(m); m->code[a].op = 0xD2; m->code[a].idx = rd_u32(&s);
            uint32_t b = push_instr(m); m->code[b].op = 0x0B; m->code[b].is_last = 1;
            e->items_start[q] = a; e->items_len[q] = 2;
          }
        }
      }
      break;
    }
    case 10: {
      uint32_t n = rd_u32(&s);
      if (n != nfunc_decl) { *err = E_MALFORMED; break; }
      m->funcs = realloc(m->funcs, sizeof(Func) * (m->nfuncs + n + 1));
      /* (all of them: a body that fails to load leaves the rest unvisited, and om_free
       * frees every function's ltypes) */
      memset(&m->funcs[m->nfuncs], 0, sizeof(Func) * (n + 1));
      for (uint32_t k = 0; k < n && !*err; k++) {
        Func *F = &m->funcs[m->nfuncs + k];
        F->type = func_types[k];
        if (F->type >= m->ntypes) { *err = E_TYPECHECK; break; }
        uint32_t blen = rd_u32(&s);
        const uint8_t *bend = s.p + blen;
        uint32_t ngroups = rd_u32(&s);
        uint32_t total = 0;
        const uint8_t *save = s.p;
        for (uint32_t g = 0; g < ngroups; g++) {
          uint32_t c = rd_u32(&s); rd_u8(&s);
          if ((uint64_t)total + c > 50000) { *err = 0x30; break; }
          total += c;
        }
        if (*err) break;
        FType *ft = &m->types[F->type];
        F->nlocals = total;
        F->ltypes = calloc(ft->np + total + 1, 1);
        memcpy(F->ltypes, ft->p, ft->np);
        s.p = save;
        uint32_t at = ft->np;
        for (uint32_t g = 0; g < ngroups; g++) {
          uint32_t c = rd_u32(&s); uint8_t t = rd_u8(&s);
          for (uint32_t q = 0; q < c; q++) F->ltypes[at++] = t;
        }
        *err = load_instr_seq(m, &s, &F->start, &F->len);
        if (!*err && s.p != bend) *err = E_MALFORMED;
      }
      m->nfuncs += n;
      break;
    }
    case 11: {
      m->ndatas = rd_u32(&s);
      m->datas = calloc(m->ndatas + 1, sizeof(Data));
      for (uint32_t k = 0; k < m->ndatas && !*err; k++) {
        Data *d = &m->datas[k];
        uint32_t flags = rd_u32(&s);
        d->mode = (flags & 1) ? 1 : 0;
        if (flags == 2) d->mem = rd_u32(&s);   /* (segment.cpp:316-323) */
        if (!(flags & 1)) *err = load_const_expr(m, &s, &d->off_start, &d->off_len);
        d->len = rd_u32(&s);
        d->bytes = malloc(d->len + 1);
        if (s.p + d->len > s.end) { *err = E_MALFORMED; break; }
        memcpy(d->bytes, s.p, d->len); s.p += d->len;
      }
      break;
    }
    case 12: rd_u32(&s); break;
    default: *err = E_MALFORMED;
    }
    if (s.err && !*err) *err = s.err;
    r.p = send;
  }
  free(func_types);
  if (!*err && m->nfuncs - m->nimported != nfunc_decl) *err = E_MALFORMED;
  for (uint32_t f = m->nimported; f < m->nfuncs && !*err; f++) *err = check_func(m, f);
  for (uint32_t k = 0; k < m->ndatas && !*err; k++)   /* an active segment's memory */
    if (m->datas[k].mode == 0) *err = mem_idx_err(m, m->datas[k].mem);
  if (*err) { om_free(m); return NULL; }
  return m;
}

void om_free(OMod *m) {
  if (!m) return;
  for (uint32_t f = 0; f < m->nfuncs; f++) free(m->funcs[f].ltypes);
  for (uint32_t k = 0; k < m->nexports; k++) free(m->exports[k].name);
  for (uint32_t k = 0; k < m->nelems; k++) { free(m->elems[k].items_start); free(m->elems[k].items_len); }
  for (uint32_t k = 0; k < m->ndatas; k++) free(m->datas[k].bytes);
  free(m->types); free(m->funcs); free(m->code); free(m->labels); free(m->tables);
  free(m->globals); free(m->exports); free(m->elems); free(m->datas);
  free(m);
}

int om_find_func(const OMod *m, const char *name, uint32_t *np, uint8_t *pt, uint32_t *nr,
                 uint8_t *rt) {
  for (uint32_t k = 0; k < m->nexports; k++) {
    if (m->exports[k].kind == 0 && !strcmp(m->exports[k].name, name)) {
      uint32_t fi = m->exports[k].idx;
      FType *t = &m->types[m->funcs[fi].type];
      if (np) *np = t->np;
      if (pt) memcpy(pt, t->p, t->np);
      if (nr) *nr = t->nr;
      if (rt) memcpy(rt, t->r, t->nr);
      return (int)fi;
    }
  }
  return -1;
}

#include "wasm_oracle_exec.inc"
