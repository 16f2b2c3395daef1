/*
 * wasm_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C restatement of the reference interpreter path (WasmEdge 0.9.1):
 *   loader      lib/loader/ast/instruction.cpp:35-116   (JumpEnd/JumpElse/IsLast)
 *   validator   lib/validator/formchecker.cpp:202-1423  (Jump descriptors, StackOffset)
 *   executor    lib/executor/engine/engine.cpp:68-1638   (dispatch loop + counting)
 *   stack       include/runtime/stackmgr.h:25-148        (16-byte ValVariant slots)
 *   memory      include/runtime/instance/memory.h:34-332 (bounds, grow, page limit)
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product (libwasmedge_batch.so) never links or calls it.
 *
 * Parity pins (see DESIGN.md "Oracle"): fib/fac example KATs (tools/wasmedge/examples),
 * mt19937 KATs (test/thread/ThreadTest.cpp:158-163), fib(30) instruction count
 * 28,271,634 (measured on the reference), node/V8 cross-checks.
 */
#ifndef WASM_ORACLE_H
#define WASM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct OMod OMod;
typedef struct OInst OInst;

/* Load + validate a module. page_limit mirrors RuntimeConfigure::MaxMemPage
 * (include/common/configure.h:123). Returns NULL and an ErrCode in *err on failure. */
OMod *om_load(const uint8_t *wasm, uint32_t len, uint32_t page_limit, int *err);
void om_free(OMod *m);

/* Function lookup by export name. Types use the wasm valtype bytes (0x7F i32 ...). */
int om_find_func(const OMod *m, const char *name, uint32_t *nparams, uint8_t *ptypes,
                 uint32_t *nresults, uint8_t *rtypes);

/* Instantiate (memory, globals, tables, elem/data init, start function). */
OInst *om_instantiate(OMod *m, int *err);
void om_inst_free(OInst *i);

/* Invoke function index fidx. Values are 16 bytes each (lo,hi u64 pairs), as
 * WasmEdge_Value's uint128 (include/api/wasmedge/wasmedge.h:39-46). Returns ErrCode
 * (0 success, 0x84.. traps). *count receives the reference-rule instruction count. */
int om_invoke(OInst *i, uint32_t fidx, const uint64_t *params, uint64_t *results,
              uint64_t *count);

/* 1 if the last om_invoke on this instance ended in Terminated (a host proc_exit; the
 * reference treats it as success, engine.cpp:62-64, with unspecified return values). */
int om_terminated(const OInst *i);

/* Gas (statistics.h:32,69-91). om_set_metering applies to instances created afterwards:
 * limit 0 = off; tab NULL + len 0 = unit costs, else len entries by OpCode, the rest 0.
 * The instance's gas total runs on from instantiation (constant expressions, start
 * function) across its invocations, like the reference VM's Statistics::CostSum.
 * om_set_cost_limit changes the limit of an existing instance. */
void om_set_metering(uint64_t limit, const uint64_t *tab, uint32_t len);
void om_set_cost_limit(OInst *i, uint64_t limit);
uint64_t om_cost_sum(const OInst *i);
/* Accept imports no test host module provides; calling one fails (test infrastructure). */
void om_set_lazy_imports(int on);

/* WASI subset of the batched path (WasmEdge_BatchInitWASI): bind wasi_snapshot_preview1
 * args/environ get+sizes, fd_write, proc_exit, sched_yield with these args/envs (shared
 * by every instance). Per instance: captured fd 1/2 bytes and the proc_exit code. */
void om_set_wasi(int on, const char *const *args, uint32_t nargs, const char *const *envs,
                 uint32_t nenvs);
/* fd_prestat_get / fd_prestat_dir_name: preopened directories ("guest:host" or one path)
 * as fds 3, 4, ... for later instantiations; an instance's own args (one Environ per VM). */
void om_set_wasi_preopens(const char *const *dirs, uint32_t n);
void om_set_instance_args(OInst *i, const char *const *args, uint32_t n);
/* WASI file/clock/random subset (wasi_fs.inc): reproducible fds, random_get and clocks
 * (seed, clock_ns), and the instance id an instance's generator is keyed on */
void om_set_wasi_deterministic(int on, uint64_t seed, uint64_t clock_ns);
void om_wasi_set_lane(OInst *i, uint32_t lane);
uint32_t om_wasi_exit_code(const OInst *i);
uint64_t om_wasi_output(const OInst *i, uint32_t fd, const uint8_t **data);

/* Tables / memories / globals provided for non-function imports (kind 1 table, 2 memory,
 * 3 global; the batched path's WasmEdge_BatchCreateWithImports), for modules loaded
 * afterwards. */
void om_clear_imports(void);
/* The TailCall proposal (return_call / return_call_indirect) for modules loaded from now
 * on; off by default (configure.h:176-182), when the loader rejects them (IllegalOpCode). */
void om_set_tail_call(int on);
void om_set_multi_memory(int on);   /* the MultiMemories proposal for modules loaded from now on */
void om_add_import(const char *mod, const char *name, uint32_t kind, uint32_t type, uint32_t mut,
                   uint32_t min, uint32_t max, int has_max, uint64_t lo, uint64_t hi);

/* Test host module "extern" (the reference API test's): the int32 an externref handle
 * points to. Table entry write (ref: function index / handle, UINT64_MAX null) and a
 * global's value bits, as the reference C API's TableInstanceSetData / GlobalInstanceGetValue. */
void om_set_extern_value(uint32_t handle, int32_t v);
int om_table_set(OInst *i, uint32_t tab, uint32_t off, uint64_t ref);
void om_global_get(const OInst *i, uint32_t g, uint64_t *lo, uint64_t *hi);

/* Linear memory 0 view and hash (hash defined in DESIGN.md, shared with the GPU). */
uint32_t om_mem_pages(const OInst *i);
const uint8_t *om_mem_data(const OInst *i);
uint64_t om_mem_hash(const OInst *i);
uint64_t om_hash_bytes(const uint8_t *data, uint64_t nbytes, uint32_t pages);

/* Batch driver (CPU baseline): one fresh instance per invocation, `threads` host
 * threads, contiguous instance-id blocks per thread. params: [n][nparams][2] u64.
 * results: [n][nresults][2]; codes/counts/hashes may be NULL. Returns wall seconds. */
double om_run_batch(OMod *m, uint32_t fidx, uint32_t n, const uint64_t *params,
                    uint64_t *results, uint8_t *codes, uint64_t *counts, uint64_t *hashes,
                    int threads);
/* om_run_batch plus mem_bytes[n]: linear-memory bytes each invocation accessed (loads,
   stores, bulk-op operands), the C3 roofline's algorithmic bytes */
double om_run_batch_mb(OMod *m, uint32_t fidx, uint32_t n, const uint64_t *params,
                       uint64_t *results, uint8_t *codes, uint64_t *counts, uint64_t *hashes,
                       uint64_t *mem_bytes, int threads);
/* om_run_batch_mb plus store_bytes[n]: the part of mem_bytes that was written (stores,
   bulk-op destinations, host-function writes) */
double om_run_batch_ms(OMod *m, uint32_t fidx, uint32_t n, const uint64_t *params,
                       uint64_t *results, uint8_t *codes, uint64_t *counts, uint64_t *hashes,
                       uint64_t *mem_bytes, uint64_t *store_bytes, int threads);

/* TEST INFRASTRUCTURE: a test host function's cost (HostFunctionBase::Cost), by import
   module / name, for instances created afterwards; mod NULL clears every cost */
void om_set_host_cost(const char *mod, const char *name, uint64_t cost);

#ifdef __cplusplus
}
#endif
#endif
