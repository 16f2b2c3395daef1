// kparams.h -- launch parameters of the batched interpreter kernel (by value).
#pragma once
#include <stdint.h>

#include "dbc.h"

struct KParams {
  // module (read-only, shared by every lane)
  const DInstr *code;
  const uint32_t *brtab;        // (target pc, tcnt) pairs
  const uint32_t *vconst;       // v128 pool
  const DFunc *funcs;           // call_indirect targets
  const uint32_t *table;        // funcref table 0 (function indices, ~0 = null)
  const uint32_t *global_init;  // initial global cells
  const uint8_t *data_pool;     // passive/active data bytes (memory.init)
  const uint32_t *data_off;
  const uint32_t *data_len;
  const void *tcode;            // threaded code for the dispatch core (tc.h), or NULL
  // per-lane state (lane-interleaved per wave)
  uint32_t *mem;                // linear memory, [wave][word][64]
  uint32_t *gstack;             // spilled frames, [wave][slot][64]
  uint32_t *lstate;             // instance state, [wave][ls_slots][64]: LS_* slots below
  uint32_t *fsave;              // frames of lanes parked at a host import, [wave][cell][64]
  uint32_t *hcall;              // [n] import being called (out) / result cells (in, ~0: done)
  uint32_t *hbuf;               // [n][hb_cells] import args (out) / results (in)
  uint32_t *hframe;             // frames in HBM, [wave][cell][64], when they exceed LDS
                                // (else NULL: frames in LDS / VGPRs)
  // per-instance inputs / outputs
  const uint32_t *params;       // [n][param_cells]
  uint32_t *results;            // [n][result_cells]
  uint8_t *status;              // [n]
  uint64_t *counts;             // [n]
  // sizes
  uint32_t n;                   // instances in this launch
  uint32_t entry_pc;
  uint32_t param_cells, result_cells;
  uint32_t global_cells, total_cells;
  uint32_t table_size;
  uint32_t mem_words;           // words per lane in the reserved layout (= rpages * 16384)
  uint32_t mlog;                // log2 of the words per interleave granule (dbc_ops.h GMem)
  uint32_t init_pages;
  uint32_t mem_max_pages;       // page limit: min(65536, the module's max, MaxMemoryPage)
                                // (memory.h:88-115 growPage)
  // Paged linear memory (DESIGN.md "Linear memory"): pages [0, rpages) of every lane live
  // in the reserved, lane-interleaved layout at `mem`; page q >= rpages of a wave lives in a
  // pool row (64 lanes x 64 KiB, same interleave) whose device address is
  // ptab[wave * ptab_w + (q - rpages)] (0 = not allocated). Only the host allocates rows;
  // a memory.grow past the wave's rows parks the lane (grow_host) for the host to do so.
  uint32_t rpages;
  const uint64_t *ptab;
  uint32_t ptab_w;
  uint32_t grow_host;           // 1: a grow past the allocated rows yields to the host
  uint32_t gs_depth;            // call-stack cells per lane
  uint32_t gs_lds;              // of which the first gs_lds live in LDS (after the frames)
  uint32_t init_dropped;        // data segments dropped after instantiation (bitmask)
  uint32_t ls_slots;            // LS_GLOBALS + global_cells
  uint32_t is_start;            // this launch runs the start function (instantiation)
  uint32_t resume;              // continue the lanes parked at a host import
  uint32_t hb_cells;
  uint64_t max_steps;           // instruction budget per instance (Interrupted, coarse)
  // gas metering (statistics.h:32,69-91): when cost_off is set, every retired wasm
  // instruction adds its cost to the lane's running total (LS_COST) and the first one
  // that would take it past cost_limit fails with CostLimitExceeded (0x03), counted.
  // cost_pool[cost_off[pc] + j] = the cost of DBC pc's first j+1 instructions
  // (Program::dops, prefix sums); cost_else = the cost of a manually counted `else`.
  uint64_t cost_limit;
  const uint32_t *cost_off;
  const uint64_t *cost_pool;
  uint64_t cost_else;
  // per-lane tables (frontend.h Program::mut_tables), else NULL / 0 and `table` serves
  uint32_t *ltab;               // [wave][tab_words][64] refs, ~0 = null
  const uint32_t *tabinfo;      // [ntables][2]: first word, capacity
  const uint32_t *elem_pool;    // element segment items (function index, ~0 = null)
  const uint32_t *elem_off, *elem_len;
  uint32_t mut_tables, ntables, tab_words;
  uint32_t ls_tab;              // LS slot of table 0's size; ls_tab + ntables: the dropped-elem
                                // mask words (32 segments each)
  uint32_t ls_drop_ext;         // LS slot of the dropped-data mask's second word (segments
                                // 32..63; LS_DROPPED holds 0..31)
  uint32_t *stop;               // host-set interrupt request (WasmEdge_BatchInterrupt)
  uint64_t max_ticks;           // wall-clock budget per wave in 100 MHz ticks
  uint64_t *stats;              // WB_STATS builds: per-wave counters (else unused)
  uint32_t sched;               // diverged waves run the lowest pc's lanes, or the largest
                                // group outside their innermost loop if it has >= sched x
                                // as many (0: min pc only)
  const uint32_t *loops;        // per pc: innermost loop (head, end), ~0 = none
  uint32_t *wave_ctr;           // persistent waves: the next wave to run (NULL: one launch
                                // wave per wave of the batch, the block's own)
  const uint32_t *wave_order;   // persistent waves: the batch waves in the order they are
                                // taken (NULL: id order) -- longest first by the last launch
  uint32_t *wave_ticks;         // persistent waves: each batch wave's run time (100 MHz ticks,
                                // or NULL)
  uint32_t simt;                // V frames + compiled runs: every running lane enters the
                                // core, whose compiled runs schedule the lanes among
                                // themselves (jit.cpp Lsched); the C++ loop only serves
                                // what the core leaves to it
  uint32_t gs_grow;             // 1: a call past gs_depth parks for the host to grow the call
                                // stack (WB_STACK_CALL) instead of trapping 0xB0
  // memories 1..n_xmem (MultiMemories): each lane's xwords words hold them back to back,
  // memory k at word xinfo[2(k - 1)], interleaved over the wave's 64 lanes in granules of
  // 4 << xlog bytes as memory 0 is (GMem: [wave][word >> xlog][64][2^xlog]); xpages[(k - 1)
  // * xstride + lane] = memory k's size, xinfo[2(k - 1) + 1] = its page limit (the
  // reservation). (A device table, not arrays in KParams: indexing those would move KParams
  // off SGPRs.)
  uint32_t *xmem;
  uint32_t *xpages;
  uint32_t *parked;             // host-mapped word: 1 when a lane parked for the host (the host
                                // then runs its service round; 0 = none parked, no round)
  const uint32_t *xinfo;
  uint32_t xwords, xstride, n_xmem, xlog;
  // 1: a table.grow past its table's capacity (tabinfo), within tlimit[t] (frontend.h
  // table_widen_limit), parks for the host to widen the tables (WB_TGROW_CALL | t) instead
  // of returning -1
  uint32_t tg_grow;
  const uint32_t *tlimit;
  // a Reset folded into this launch (batch_kernel.hip fused_reset): the memory image, the
  // rows a Reset covers, and the instance state's initial words (StateInit)
  uint32_t rf_on, rf_image_words, rf_init_words, rf_init_pages, rf_init_dropped;
  const uint32_t *rf_image, *rf_global_init;
  uint64_t rf_init_cost;
};

// Per-lane instance state that persists across invocations until the next Reset (the
// reference keeps it in ModuleInstance / MemoryInstance / GlobalInstance): memory size,
// dropped data segments, instantiation status (a trapped start function fails the
// instance, module.cpp:160-170), the resume point of a lane parked at a host import
// (pc, call-stack depth, arg/result cell; pc ~0 = not parked), the write mark, the gas
// total, then the global cells,
// then (per-lane tables only) each table's size and the dropped-elem-segment mask.
#define LS_PAGES 0u
#define LS_DROPPED 1u
#define LS_ISTATUS 2u
#define LS_RPC 3u
#define LS_GSP 4u
#define LS_HBASE 5u
#define LS_HWM 6u      // one past the highest linear-memory byte written since instantiation
#define LS_COST 7u     // 2 slots: the instance's running gas total (lo, hi), kept from
                       // instantiation on like the reference VM's Statistics::CostSum
#define LS_GLOBALS 9u
