// frontend.h -- host-side module decoder, validator and DBC lowering.
//
// Replaces, for the batched path, what the reference does in
//   lib/loader/loader.cpp:64-163 + lib/loader/ast/*.cpp   (decode, JumpEnd/JumpElse)
//   lib/validator/validator.cpp:19-117 + formchecker.cpp   (type check, branch resolution)
//   lib/executor/instantiate/module.cpp:16-172              (per-instance initial state)
// producing a Program: register-form device bytecode + the module image every lane
// starts from (memory pages, data segments, globals, tables).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "dbc.h"

namespace wb {

enum ValT : uint8_t { I32 = 0x7F, I64 = 0x7E, F32 = 0x7D, F64 = 0x7C, V128 = 0x7B,
                      FUNCREF = 0x70, EXTERNREF = 0x6F, UNKNOWN = 0 };

inline uint32_t cells_of(uint8_t t) { return t == I64 || t == F64 ? 2 : (t == V128 ? 4 : 1); }

struct FuncType {
  std::vector<uint8_t> params, results;
  bool operator==(const FuncType &o) const { return params == o.params && results == o.results; }
};

struct DataSeg {
  bool active = true;
  uint32_t mem = 0;                   // the memory an active segment initialises
  uint32_t offset = 0;
  std::vector<uint8_t> bytes;
};

struct TableInfo {
  uint8_t type = FUNCREF;
  uint32_t min = 0, max = 0;
  bool has_max = false;
};

struct ElemSeg {
  bool active = false, declarative = false;
  uint8_t type = FUNCREF;
  uint32_t table = 0, offset = 0;
  std::vector<uint32_t> items;        // function index per item, 0xFFFFFFFF = null ref
};

// Per-lane table capacity beyond `min` a table starts with when it has no (or a larger)
// max; a table.grow past it widens every lane's table (hostcall.cpp widen_tables).
constexpr uint32_t kTableGrowLimit = 4096;
// The most entries a table can widen to per lane (with its max, if smaller): table.grow
// past it returns -1, as at the reference's Refs vector failing to grow (table.h:59-72).
constexpr uint32_t kTableWidenMax = 1u << 24;
inline uint32_t table_widen_limit(const struct TableInfo &T) {
  return T.has_max && T.max < kTableWidenMax ? T.max : kTableWidenMax;
}
// memories past the first a module may have (MultiMemories)
constexpr uint32_t kMaxXMem = 7;

struct ExportFunc {
  std::string name;
  uint32_t func;
};

struct FuncInfo {
  uint32_t type = 0;
  bool imported = false;
  std::string import_module, import_name;
  uint32_t entry_pc = 0, body_pc = 0;
  uint32_t param_cells = 0, local_cells = 0, frame_cells = 0;
  std::vector<uint8_t> local_types;   // declared locals (not params)
  uint32_t code_off = 0, code_len = 0; // byte range of the body in the binary
};

struct Program {
  // module
  std::vector<FuncType> types;
  std::vector<uint32_t> type_canon;    // type index -> canonical structural id
  std::vector<FuncInfo> funcs;
  uint32_t n_imported = 0;
  std::vector<ExportFunc> exports;
  std::vector<ExportFunc> table_exports, global_exports;   // name -> table / global index
  bool has_mem = false;
  uint32_t mem_min = 0, mem_max = 65536;
  bool mem_has_max = false;
  // memories 1.. (the MultiMemories proposal; every memory instruction on them runs in the
  // per-lane step, batch_kernel.hip "extra memories"): limits as memory 0's
  struct MemLimits { uint32_t min = 0, max = 65536; bool has_max = false; };
  std::vector<MemLimits> xmems;
  std::vector<DataSeg> datas;
  std::vector<uint8_t> global_types;
  std::vector<uint8_t> global_mut;
  std::vector<uint32_t> global_cell;   // first cell of each global
  std::vector<uint32_t> global_init;   // initial cell values, G cells
  uint32_t global_cells = 0;           // G = frame base
  std::vector<uint32_t> table0;        // funcref table 0 (immutable), 0xFFFFFFFF = null
  uint32_t ntables = 0;
  std::vector<TableInfo> tables;
  std::vector<ElemSeg> elems;
  // Per-lane tables (tableInstr.cpp): set when the code mutates a table (table.set/grow/
  // fill/copy/init, elem.drop), or has several tables or an externref table. Then every
  // lane owns tab_words words (tables back to back, tabinfo = {first word, capacity} per
  // table) initialised from tab_image, sizes and dropped elem segments live in its
  // instance state, and table0 is unused.
  bool mut_tables = false;
  std::vector<uint32_t> tab_image, tabinfo;
  std::vector<uint32_t> elem_pool, elem_off, elem_len;
  uint32_t tab_words = 0;
  // dropped element segments at instantiation (active and declarative ones, elem.cpp), a
  // bit per segment, 32 per word; per-lane tables keep these words in the instance state
  std::vector<uint32_t> init_edropped;
  int64_t start_func = -1;
  // lowered code
  std::vector<DInstr> code;
  // per DBC instruction: the wasm opcodes (reference OpCode numbering, 0xFCxx / 0xFDxx for
  // prefixed ones) of the instructions it retires, in execution order -- its `cnt`
  // entries, the last `post` of them after the main op. A taken branch with tcnt = -k
  // retires its landing instruction's list from entry k on; tcnt = +1 (if-false to an
  // else arm) also retires an `else` (controlInstr.cpp:23-28). Cost tables price these.
  std::vector<std::vector<uint16_t>> dops;
  std::vector<uint16_t> init_ops;      // instructions of every constant expression (counted
                                       // and priced by instantiation, before the start function)
  std::vector<uint32_t> brtab;         // pairs (target pc, tcnt as int32)
  std::vector<uint32_t> loops;         // per pc: (head, end) of the innermost loop around
                                       // it (a backward branch end -> head), ~0 if none
  std::vector<uint32_t> vconst;        // v128 pool, 4 words per entry
  uint32_t frame_cells = 0;            // max over functions (excluding globals)
  uint32_t total_cells() const { return global_cells + frame_cells; }
  uint32_t max_wasm_instrs_per_dispatch = 0;
  // metered lowering: global.set never retargets its producer, so a cost-limit trap
  // between a value and its global.set leaves the global unwritten as in the reference
  bool exact_globals = false;
  // the TailCall proposal (return_call / return_call_indirect) is enabled; off, they fail
  // to load with IllegalOpCode like the reference's default (loader/ast/instruction.cpp:903-907)
  bool tail_call = false;
  // the MultiMemories proposal: several memories and memory indices in memory
  // instructions (instruction.cpp:144-156, 374-389); off, a second memory fails with
  // MultiMemories (0x51, validator.cpp:107-113)
  bool multi_memory = false;
  // some load/store address depends on per-instance data (a parameter, a loaded value, a
  // global): the batch then interleaves memory in 128-byte granules (batch_api.cpp)
  bool divergent_mem = false;
  // the same for a memory past the first (its layout is fixed; only the trip-mode choice
  // reads it)
  bool divergent_xmem = false;
};

// A table, memory or global import the embedder provides (WasmEdge_BatchImport). Every
// instance gets a copy of its own, as each reference VM gets its own import object: a
// memory of `min` zeroed pages, a table of `min` null references, a global = value.
struct HostImport {
  std::string module, name;
  uint8_t kind = 0;                  // 1 table, 2 memory, 3 global (ExternalType)
  uint8_t type = 0;                  // table: reference type; global: value type
  bool mut = false;                  // global
  uint32_t min = 0, max = 0;         // table / memory limits
  bool has_max = false;
  uint32_t value[4] = {0, 0, 0, 0};  // global: its value as cells
};

// Load + validate + lower. Returns empty string on success, else an error message;
// *errcode receives the reference ErrCode byte (include/common/enum.inc). Non-function
// imports resolve against `imports` like instantiate/import.cpp (UnknownImport 0x62,
// IncompatibleImportType 0x61).
std::string load_program(const uint8_t *wasm, size_t len, Program &out, uint8_t *errcode,
                         bool exact_globals = false,
                         const std::vector<HostImport> *imports = nullptr, bool tail_call = false,
                         bool multi_memory = false);

int find_export(const Program &p, const std::string &name);

// Gas metering tables for a cost table `tab` (65536 entries, indexed by the reference's
// OpCode; statistics.h:32 CostTab): off[pc] / pool hold each DBC's prefix sums of the
// costs of the instructions it retires (KParams::cost_pool); the return value is the gas
// instantiation's constant expressions spend, priced one by one against `limit` like
// Statistics::addCost (*exceeded: one of them fails with CostLimitExceeded).
uint64_t build_cost_pool(const Program &p, const uint64_t *tab, uint64_t limit,
                         std::vector<uint32_t> &off, std::vector<uint64_t> &pool, bool *exceeded);

const char *dop_name(uint16_t op);

}  // namespace wb
