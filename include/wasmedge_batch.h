/*
 * wasmedge_batch.h -- C ABI of the MI355X batched WebAssembly interpreter.
 *
 * A batched entry placed BESIDE the reference's WasmEdge_VMExecute
 * (include/api/wasmedge/wasmedge.h:3301-3303, lib/api/wasmedge.cpp:2687-2698): one
 * validated module, N independent instances, one GPU lane each.  Conventions follow the
 * reference C API (include/api/wasmedge/wasmedge.h:39-60):
 *   - values are WasmEdge_Value {uint128_t Value; enum WasmEdge_ValType Type};
 *   - errors are returned by value as WasmEdge_Result{uint8_t Code} holding the
 *     reference ErrCode byte (include/common/enum.inc:573-749);
 *   - buffers are caller-owned; surplus returns are dropped, a ReturnLen shortfall is
 *     silent (lib/api/wasmedge.cpp:245-255 fillWasmEdge_ValueArr);
 *   - a NULL context gives WrongVMWorkflow (0x04) (lib/api/wasmedge.cpp:266-277);
 *   - contexts returned by *Create are owned by the caller and freed by *Delete.
 * Per-instance outcomes (traps) are reported per lane with the reference trap codes
 * (0x84..0x8E), never through the call-level result.
 *
 * Plain C types only; no torch/HIP types cross this boundary.
 */
#ifndef WASMEDGE_BATCH_H
#define WASMEDGE_BATCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef WASMEDGE_C_API_H /* use the reference's definitions when its header is included */
typedef unsigned __int128 uint128_t;
enum WasmEdge_ValType {
  WasmEdge_ValType_I32 = 0x7FU,
  WasmEdge_ValType_I64 = 0x7EU,
  WasmEdge_ValType_F32 = 0x7DU,
  WasmEdge_ValType_F64 = 0x7CU,
  WasmEdge_ValType_V128 = 0x7BU,
  WasmEdge_ValType_FuncRef = 0x70U,
  WasmEdge_ValType_ExternRef = 0x6FU
};
typedef struct WasmEdge_Value {
  uint128_t Value;
  enum WasmEdge_ValType Type;
} WasmEdge_Value;
typedef struct WasmEdge_String {
  uint32_t Length;
  const char *Buf;
} WasmEdge_String;
typedef struct WasmEdge_Result {
  uint8_t Code;
} WasmEdge_Result;
#endif

#define WASMEDGE_BATCH_API __attribute__((visibility("default")))

/* Per-instance status byte (PerInstance[i]) beyond the reference trap codes. */
#define WASMEDGE_BATCH_OK 0x00u
#define WASMEDGE_BATCH_INTERRUPTED 0x07u      /* ErrCode::Interrupted: step/time limit */
#define WASMEDGE_BATCH_STACK_EXHAUSTED 0xB0u  /* device call stack full */
#define WASMEDGE_BATCH_HOST_CALL 0xB1u        /* reached a host import no host function is bound to */

typedef struct WasmEdge_BatchConfigure {
  /* Page limit per instance: RuntimeConfigure::MaxMemPage (include/common/configure.h:
   * 112-123; 0 = its default, 65536). memory.grow returns -1 past it, past the module's
   * declared maximum and past 65536 pages, or when the device has no memory left for the
   * new pages -- MemoryInstance::growPage (include/runtime/instance/memory.h:87-115) with
   * Allocator::resize failing (lib/system/allocator.cpp:101-129). Pages are committed on
   * demand, as the reference's mmap'd reservation is: see MemoryReservePages. A module
   * whose initial size exceeds a non-zero limit fails WasmEdge_BatchCreate with
   * MemoryOutOfBounds (0x88): the reference allocates no memory for it (memory.h:46-51). */
  uint32_t MaxMemoryPage;
  /* Device call-stack depth per instance in 32-bit cells. 0 (the default): the stack
   * starts at 4096 cells and grows on demand, as the reference's StackManager vectors do
   * (include/runtime/stackmgr.h:44-47) -- a call past it parks the instance, the stack
   * doubles between launches and the call runs again (counted once); only when the device
   * has no memory left for it does a call end the instance with 0xB0. Non-zero: a fixed
   * bound, 0xB0 past it. */
  uint32_t CallStackCells;
  /* Instruction budget per instance (0 = unlimited; counted in the reference's
   * Statistics units; checked every scheduler round, and a device-side core call never
   * runs a lane more than one compiled run past its remaining budget) and wall-clock limit per
   * launch in seconds (0 = 600); exceeding either marks the instance Interrupted (0x07),
   * mirroring the reference's cost limit / StopToken (statistics.h:69-91,
   * helper.cpp:24-27). */
  uint64_t MaxSteps;
  double TimeLimitSeconds;
  /* HIP device ordinal (-1 = the current device). */
  int32_t DeviceOrdinal;
  /* Gas limit per instance (StatisticsConfigure::setCostLimit, statistics.h:32,69-91;
   * 0 = no metering). Every wasm instruction adds its cost to the instance's running
   * total; the first one that would take the total past CostLimit fails with
   * CostLimitExceeded (0x03), counted but not executed (engine.cpp:1616-1630). The total
   * starts at instantiation, whose constant expressions and start function spend gas too,
   * and runs on across Execute/Run calls until BatchReset, like the reference VM's
   * Statistics::CostSum. Metered contexts run the compiled runs, which price themselves
   * exactly, and the per-lane step (no SIMT scheduling). */
  uint64_t CostLimit;
  /* Host threads serving lanes parked at host imports. 0 or 1: one thread, host
   * functions are called one at a time. More: waves are spread over that many threads
   * (a wave's lanes stay on one), so host functions must then be reentrant, as the
   * reference's are under concurrent VM::execute. */
  uint32_t HostThreads;
  /* Cost per instruction, indexed by the reference's OpCode (include/common/enum.inc:
   * one-byte opcodes, 0xFCxx, 0xFDxx): CostTableLen entries, the rest 0 -- the batched
   * WasmEdge_StatisticsSetCostTable (lib/api/wasmedge.cpp:878-882, statistics.h:59-66).
   * NULL with length 0: the default table, every instruction costs 1. Copied at
   * BatchCreate. */
  const uint64_t *CostTable;
  uint32_t CostTableLen;
  /* Bytes per granule in which the device interleaves the linear memories of a wave's 64
   * instances (4, 8, ..., 128; 0 = chosen: 4 when the module's load/store addresses are the
   * same in every instance; when an address may depend on per-instance data, a layout trial
   * decides from measured throughput -- the first Run is an unmeasured warm-up at 128, the
   * second is measured at 128, the next Reset re-lays memory in 4-byte words and the Run
   * after it is measured again; 4 stays if at least 10% faster per wasm instruction on the
   * same function, else the following Reset goes back to 128 (WB_GRANULE_TRIAL=0: 128, no
   * trial). The shards of a multi-device batch take the first shard's verdict.) Layout
   * only: results never depend on it. WasmEdge_BatchGetMemoryGranule reports the layout in
   * use. */
  uint32_t MemoryGranule;
  /* The TailCall proposal (return_call, return_call_indirect; WasmEdge_ConfigureAddProposal
   * (Conf, WasmEdge_Proposal_TailCall), include/common/configure.h:176-182 leaves it off):
   * 0 = off, the opcodes fail BatchCreate with IllegalOpCode (0x37) as in the reference's
   * loader. On: a tail call reuses the caller's frame, so tail recursion never exhausts the
   * device call stack; a host import in tail position runs on the yield path and its results
   * return from the caller (DESIGN.md "Tail calls"). */
  uint32_t TailCall;
  /* Layout of linear memory on the device (results never depend on it). The first
   * MemoryReservePages pages of every instance are allocated up front in the lane-
   * interleaved layout every execution path addresses directly; pages an instance grows
   * past them are committed on demand in 4 MiB rows (the page for all 64 instances of a
   * wave) and reached through a page table by the per-lane step, more slowly. 0 = the
   * module's initial size, raised toward the page limit while the whole batch's
   * reservation stays within min(16 GiB, a quarter of the device's free memory); modules
   * without memory.grow reserve their initial size. Clamped to [initial size, limit]. After
   * a run whose instances grew past it, the next BatchReset re-lays memory with the largest
   * size they reached in the reserved layout (WasmEdge_BatchGetReservedPages), so later runs
   * address every page directly. */
  uint32_t MemoryReservePages;
  /* Cap on the device memory committed for grown pages (bytes; 0 = until hipMalloc fails).
   * A grow that would need more returns -1. */
  uint64_t MemoryPoolBytes;
  /* Devices the batch spreads over from this one process (SURVEY.md 8(b) NumDevices, 8(e)).
   * DeviceCount 0 or 1: one device, DeviceOrdinal. More: Devices[0..DeviceCount) are HIP
   * ordinals -- a device may repeat (several shards on one device) -- and instance ids go to
   * them by Partition: WASMEDGE_BATCH_PARTITION_BLOCKS, contiguous blocks of whole waves, or
   * WASMEDGE_BATCH_PARTITION_INTERLEAVE, id mod DeviceCount (evens out work that varies
   * with the id). Every call then drives every shard -- one host thread and one stream per
   * shard, no collective -- and gathers per-instance outputs into the caller's
   * [NumInstances] arrays in instance order (WasmEdge_BatchPlacement gives the map).
   * Results never depend on it; like the reference's concurrent VM::execute
   * (include/vm/vm.h:137-141), host functions are called from one shard at a time unless
   * HostThreads > 1. */
  const int32_t *Devices;
  uint32_t DeviceCount;
  uint32_t Partition;
  /* The MultiMemories proposal (WasmEdge_ConfigureAddProposal(Conf,
   * WasmEdge_Proposal_MultiMemories), include/common/enum.inc:555; off by default,
   * configure.h:176-182): 0 = off, a second memory fails BatchCreate with MultiMemories
   * (0x51, validator.cpp:107-113). On: several memories (defined or imported) and memory
   * indices in loads, stores, memory.size/grow/fill/copy/init and data segments, read as
   * the reference reads them (a memarg's index after its offset, instruction.cpp:144-156).
   * Memory 0 keeps every execution path; instructions on the other memories run in the
   * per-lane step, on memories reserved whole per instance (their initial size, or up to
   * their limit as far as min(4 GiB, free/8) per batch goes when the module grows them; a
   * grow past that returns -1). WasmEdge_BatchGetMemory / the memory hash cover memory 0. */
  uint32_t MultiMemories;
  /* Pages reserved per instance for each memory past the first that the module grows
   * (0 = chosen as above: the page limit as far as min(4 GiB, free/8) for the whole batch
   * goes -- with tens of thousands of instances that can be few or none, and then
   * memory.grow on it returns -1 where the reference's would succeed). Clamped to [initial
   * size, limit]; BatchCreate fails with RuntimeError when the batch does not fit.
   * WasmEdge_BatchGetExtraMemoryPages reports the reservation in use. */
  uint32_t ExtraMemoryReservePages;
  /* Cap on the device memory the call stack may grow to when CallStackCells is 0 (bytes;
   * 0 = an eighth of the device's memory). Past it a call ends the instance with 0xB0.
   * Each BatchReset returns the stack to its first depth. */
  uint64_t CallStackMaxBytes;
} WasmEdge_BatchConfigure;

#define WASMEDGE_BATCH_PARTITION_BLOCKS 0u
#define WASMEDGE_BATCH_PARTITION_INTERLEAVE 1u

/* Where instance Inst of a NumInstances-instance batch over DeviceCount devices runs: the
 * index into Devices (*Shard) and its lane on that device (*Local). No device is touched.
 * WrongVMWorkflow (0x04) for Inst >= NumInstances, DeviceCount 0 or an unknown Partition. */
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchPlacement(uint32_t NumInstances, uint32_t DeviceCount,
                                                          uint32_t Partition, uint32_t Inst,
                                                          uint32_t *Shard, uint32_t *Local);

#ifdef WASMEDGE_C_API_H
/* The reference's configuration object as a batch configuration (header-inline: needs the
 * reference's wasmedge.h included first). It carries over what the reference's
 * WasmEdge_ConfigureContext decides for the interpreter path: the page limit
 * (WasmEdge_ConfigureGetMaxMemoryPage, wasmedge.h:560; RuntimeConfigure::MaxMemPage,
 * configure.h:112-123) and the TailCall and MultiMemories proposals
 * (WasmEdge_ConfigureHasProposal, wasmedge.h:495; off by default, configure.h:176-182).
 * The proposals on by default (SIMD, bulk memory, reference types, multi-value, sign
 * extension, saturating conversions, mutable globals) are always on in the batched path.
 * Statistics: instruction counts are always reported;
 * cost metering is set through CostLimit / CostTable (the reference keeps those on its
 * StatisticsContext). Fields this does not set keep the caller's values; a NULL Conf
 * leaves the reference defaults (MaxMemoryPage 0 = 65536, TailCall and MultiMemories off). */
static inline void WasmEdge_BatchConfigureFromContext(const WasmEdge_ConfigureContext *Conf,
                                                      WasmEdge_BatchConfigure *Out) {
  if (!Out) return;
  if (!Conf) {
    Out->MaxMemoryPage = 0;
    Out->TailCall = 0;
    Out->MultiMemories = 0;
    return;
  }
  Out->MaxMemoryPage = WasmEdge_ConfigureGetMaxMemoryPage(Conf);
  Out->TailCall = WasmEdge_ConfigureHasProposal(Conf, WasmEdge_Proposal_TailCall) ? 1u : 0u;
  Out->MultiMemories = WasmEdge_ConfigureHasProposal(Conf, WasmEdge_Proposal_MultiMemories) ? 1u : 0u;
}
#endif

typedef struct WasmEdge_BatchContext WasmEdge_BatchContext;

/* Load + validate + lower `WasmBuf`, allocate device state for NumInstances instances
 * and instantiate them (BatchReset). Replaces VM::loadWasm/validate/instantiate
 * (lib/vm/vm.cpp) for the batch. Returns NULL on failure with the ErrCode in *Res (may
 * be NULL). */
WASMEDGE_BATCH_API WasmEdge_BatchContext *
WasmEdge_BatchCreate(const WasmEdge_BatchConfigure *Conf, const uint8_t *WasmBuf,
                     uint32_t WasmLen, uint32_t NumInstances, WasmEdge_Result *Res);

/* A table, memory or global the embedder provides for the module's imports of that
 * kind -- the batched form of creating it (WasmEdge_TableInstanceCreate /
 * MemoryInstanceCreate / GlobalInstanceCreate, wasmedge.h) and adding it to an import
 * object (WasmEdge_ImportObjectAddTable/AddMemory/AddGlobal). Every instance gets a copy
 * of its own, as each reference VM has its own import object: a memory of Min zeroed
 * pages, a table of Min null references, a global holding Value. Matching follows
 * lib/executor/instantiate/import.cpp: an import with no provider fails with UnknownImport
 * (0x62); a provider of another reference / value type or mutability, or whose limits do
 * not fit the import's (Min >= the import's min; a Max when the import has one, no larger),
 * fails with IncompatibleImportType (0x61). Function imports bind later, through
 * WasmEdge_BatchAddHostFunction / WasmEdge_BatchInitWASI. */
#define WASMEDGE_BATCH_IMPORT_TABLE 1u
#define WASMEDGE_BATCH_IMPORT_MEMORY 2u
#define WASMEDGE_BATCH_IMPORT_GLOBAL 3u
typedef struct WasmEdge_BatchImport {
  WasmEdge_String ModuleName;
  WasmEdge_String ExternalName;
  uint32_t Kind;                /* WASMEDGE_BATCH_IMPORT_* (the reference ExternalType) */
  uint32_t Min, Max;            /* table / memory limits */
  uint32_t HasMax;
  enum WasmEdge_ValType Type;   /* table: FuncRef / ExternRef; global: its value type */
  uint32_t Mutable;             /* global: 1 = var */
  WasmEdge_Value Value;         /* global: its initial value (a funcref is a function
                                   index of the module, an externref any 64-bit value,
                                   null 0xFFFFFFFF) */
} WasmEdge_BatchImport;

/* WasmEdge_BatchCreate with the module's table / memory / global imports provided. */
WASMEDGE_BATCH_API WasmEdge_BatchContext *
WasmEdge_BatchCreateWithImports(const WasmEdge_BatchConfigure *Conf, const uint8_t *WasmBuf,
                                uint32_t WasmLen, uint32_t NumInstances,
                                const WasmEdge_BatchImport *Imports, uint32_t ImportLen,
                                WasmEdge_Result *Res);

/* Run `FuncName` on every instance (one instance per lane). Instance state -- linear
 * memory and its size, globals, dropped data segments -- persists from one Execute/Run
 * to the next until BatchReset, as an instantiated module does in the reference VM.
 * Params: [NumInstances][ParamLen] row-major; Returns: [NumInstances][ReturnLen].
 * PerInstance[i]: 0 ok, else trap/status code. InstrCounts[i]: the reference's
 * instruction count (include/common/statistics.h:44). Either may be NULL.
 * Mirrors WasmEdge_VMExecute (wasmedge.h:3301) per instance. */
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchExecute(WasmEdge_BatchContext *Cxt, const WasmEdge_String FuncName,
                      const WasmEdge_Value *Params, const uint32_t ParamLen,
                      WasmEdge_Value *Returns, const uint32_t ReturnLen,
                      uint8_t *PerInstance, uint64_t *InstrCounts);

/* SURVEY.md §8(b)'s form of the same call: the per-instance outcome as a WasmEdge_Result
 * each (Code = the status byte above). WasmEdge_Result is one byte (wasmedge.h:55-60), so
 * an array of them is the status array itself. */
typedef char WasmEdge_BatchResultIsOneByte[sizeof(WasmEdge_Result) == 1 ? 1 : -1];
static inline WasmEdge_Result
WasmEdge_BatchExecuteResults(WasmEdge_BatchContext *Cxt, const WasmEdge_String FuncName,
                             const WasmEdge_Value *Params, const uint32_t ParamLen,
                             WasmEdge_Value *Returns, const uint32_t ReturnLen,
                             WasmEdge_Result *PerInstance, uint64_t *InstrCounts) {
  return WasmEdge_BatchExecute(Cxt, FuncName, Params, ParamLen, Returns, ReturnLen,
                               (uint8_t *)PerInstance, InstrCounts);
}

/* Ask a running BatchExecute/BatchRun on this context to stop (any thread): every
 * instance still running ends with Interrupted (0x07) at the next scheduler round (the
 * flag is read every round; a core call runs at most 2^20 instructions), like the
 * reference's StopToken / async cancel (helper.cpp:24-27, include/common/async.h:73-77).
 * The request is cleared when the next Run starts. */
WASMEDGE_BATCH_API void WasmEdge_BatchInterrupt(WasmEdge_BatchContext *Cxt);

/* Staged form of BatchExecute, for callers that keep inputs resident on the device
 * and time the interpreter alone (bench.py):
 *   SetArgs  -> resolve FuncName, check types (FuncSigMismatch), upload params
 *   Reset    -> fresh instances: memory image, globals, then the start function
 *               (lib/executor/instantiate/module.cpp:16-172); a lane whose start
 *               function traps reports that trap from every later Run.
 *               *KernelSeconds = the reset kernels' time; NULL: Reset does not wait
 *               for them (without a start function), the next Run orders after them
 *   Run      -> launch the interpreter; *KernelSeconds = HIP-event time on the
 *               library's stream (may be NULL)
 *   Results  -> copy returns / statuses / counts back. */
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchSetArgs(WasmEdge_BatchContext *Cxt, const WasmEdge_String FuncName,
                      const WasmEdge_Value *Params, const uint32_t ParamLen);
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchReset(WasmEdge_BatchContext *Cxt,
                                                       double *KernelSeconds);
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchRun(WasmEdge_BatchContext *Cxt,
                                                     double *KernelSeconds);
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchResults(WasmEdge_BatchContext *Cxt, WasmEdge_Value *Returns,
                      const uint32_t ReturnLen, uint8_t *PerInstance, uint64_t *InstrCounts);

/* ---- host functions (the yield path) --------------------------------
 * A lane that calls an imported function parks on the device; BatchRun / BatchReset then
 * call the host function registered for that import on the CPU, once per parked lane,
 * write its results back and resume the lanes, until none is parked -- the batched form
 * of the reference's host-function call (lib/executor/helper.cpp:35-97,
 * include/runtime/hostfunc.h:25-40). The signature mirrors WasmEdge_HostFunc_t
 * (include/api/wasmedge/wasmedge.h:2269-2271); MemCxt is the calling instance's memory.
 * A non-zero Result ends that instance with the code in PerInstance (Terminated 0x01,
 * as from proc_exit, ends it "successfully" with zeroed returns; engine.cpp:62-64). An
 * import without a registered function ends the instance with 0xB1. */
typedef struct WasmEdge_BatchMemoryContext WasmEdge_BatchMemoryContext;
typedef WasmEdge_Result (*WasmEdge_BatchHostFunc_t)(void *Data,
                                                    WasmEdge_BatchMemoryContext *MemCxt,
                                                    const WasmEdge_Value *Params,
                                                    WasmEdge_Value *Returns);
/* Bind `Func` to every import named ModuleName.FuncName (WasmEdge_ImportObjectAddFunction,
 * wasmedge.h:2814). Register before the first Run (and before Reset when the start
 * function calls imports). */
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchAddHostFunction(WasmEdge_BatchContext *Cxt, const WasmEdge_String ModuleName,
                              const WasmEdge_String FuncName, WasmEdge_BatchHostFunc_t Func,
                              void *Data);
/* The same with the host function's gas cost: the Cost of WasmEdge_FunctionInstanceCreate
 * (Type, Func, Data, Cost) (include/api/wasmedge/wasmedge.h:2324; HostFunctionBase::Cost,
 * include/runtime/hostfunc.h:28-46). In a metered context (CostLimit) every call adds Cost
 * to the instance's gas total before the function runs; a call that would take the total
 * past CostLimit ends the instance with CostLimitExceeded (0x03) instead -- the call
 * instruction counted, the host function not run, the total unchanged -- as
 * Stat->addCost(HostFunc.getCost()) does (lib/executor/helper.cpp:59-64). The built-in WASI
 * functions cost 0, as the reference's do (include/host/wasi/wasibase.h:15). */
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchAddHostFunctionWithCost(WasmEdge_BatchContext *Cxt, const WasmEdge_String ModuleName,
                                      const WasmEdge_String FuncName, WasmEdge_BatchHostFunc_t Func,
                                      void *Data, uint64_t Cost);
/* Inside a host function: the calling instance and its memory
 * (WasmEdge_MemoryInstanceGetData / SetData, wasmedge.h:2552-2569). */
WASMEDGE_BATCH_API uint32_t
WasmEdge_BatchMemoryGetInstance(const WasmEdge_BatchMemoryContext *MemCxt);
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchMemoryGetData(const WasmEdge_BatchMemoryContext *MemCxt, uint8_t *Data,
                            const uint32_t Offset, const uint32_t Length);
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchMemorySetData(WasmEdge_BatchMemoryContext *MemCxt, const uint8_t *Data,
                            const uint32_t Offset, const uint32_t Length);

/* ---- built-in WASI subset (wasi_snapshot_preview1) on the yield path -------------------
 * Binds the module's imports args_get, args_sizes_get, environ_get, environ_sizes_get,
 * fd_write, proc_exit and sched_yield (those with the WASI signature) to host functions
 * inside the library, as WasmEdge_ImportObjectCreateWASI / InitWASI would
 * (include/api/wasmedge/wasmedge.h:2719-2754, lib/host/wasi/wasifunc.cpp), plus
 * fd_prestat_get and fd_prestat_dir_name. Args/Envs are shared by every instance unless an
 * instance has its own args (WasmEdge_BatchWASISetInstanceArgs). fd_write to fd 1 / 2 is
 * captured per instance (fd 0 gives NOTCAPABLE, other fds BADF); proc_exit records the exit code
 * and ends the instance with Terminated (0x01). Calling it again re-initialises the
 * environment and clears the captured output and exit codes. Other WASI imports stay
 * unbound (0xB1 when reached) unless registered with WasmEdge_BatchAddHostFunction. */
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchInitWASI(WasmEdge_BatchContext *Cxt, const char *const *Args, const uint32_t ArgLen,
                       const char *const *Envs, const uint32_t EnvLen);
/* The same with preopened directories, as WasmEdge_ImportObjectInitWASI's Preopens
 * (wasmedge.h:2739-2742): "guest:host" or one path for both; they become fds 3, 4, ... in
 * the order given (environ.cpp:54-93), named by VINode::canonicalGuest, with the
 * reference's rights, and behave as a read-only mount (N instances share the host
 * directory): path_open, fd_read, fd_seek, fd_tell, fd_close, fd_fdstat_get,
 * fd_filestat_get, path_filestat_get, fd_prestat_get / _dir_name work on them, an open that
 * would create, truncate or write fails with ROFS. A file is read whole when an instance
 * first opens it. Also bound: clock_time_get, clock_res_get, random_get,
 * fd_fdstat_set_flags (wasmedge_amd/csrc/wasi_impl.h lists each with its reference
 * lines). */
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchInitWASIWithPreopens(WasmEdge_BatchContext *Cxt, const char *const *Args,
                                   const uint32_t ArgLen, const char *const *Envs,
                                   const uint32_t EnvLen, const char *const *Preopens,
                                   const uint32_t PreopenLen);
/* Instance Inst's own command line (args_get / args_sizes_get), in place of the shared Args:
 * the reference builds one Environ per VM (environ.cpp:95-98), so N instances with their
 * own arguments are N VMs with their own WASI modules. Call after WasmEdge_BatchInitWASI
 * (which clears every instance's own args). */
/* Reproducible WASI: instance i's new fd numbers and random_get bytes come from a
 * generator seeded by (Seed, i) -- the reference draws both from std::random_device
 * (environ.h:834-850, 1096-1108), and so does this library by default -- and every clock
 * reads ClockNs, advancing 1 us per call of the instance (clock_res_get: 1 ns). Call after
 * the InitWASI call it applies to; it also resets the instances' fd tables. */
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchWASISetDeterministic(WasmEdge_BatchContext *Cxt, uint64_t Seed, uint64_t ClockNs);
WASMEDGE_BATCH_API WasmEdge_Result
WasmEdge_BatchWASISetInstanceArgs(WasmEdge_BatchContext *Cxt, uint32_t Inst,
                                  const char *const *Args, const uint32_t ArgLen);
/* proc_exit code of instance Inst (0 if it never called it; WasmEdge_ImportObjectWASIGetExitCode,
 * wasmedge.h:2754). */
WASMEDGE_BATCH_API uint32_t WasmEdge_BatchWASIGetExitCode(const WasmEdge_BatchContext *Cxt,
                                                          uint32_t Inst);
/* Bytes instance Inst wrote to fd 1 (stdout) or 2 (stderr); copies at most Len of them into
 * Buf (may be NULL) and returns the total size. */
WASMEDGE_BATCH_API uint32_t WasmEdge_BatchWASIGetOutput(const WasmEdge_BatchContext *Cxt,
                                                        uint32_t Inst, uint32_t Fd, uint8_t *Buf,
                                                        uint32_t Len);

/* Each instance's gas total (WasmEdge_StatisticsGetTotalCost, wasmedge.h): Costs[N];
 * all 0 when the context does not meter. */
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchGetTotalCosts(WasmEdge_BatchContext *Cxt,
                                                               uint64_t *Costs);

/* Straight-line runs of the module that the context compiled to machine code for the
 * V-frame threaded core (DESIGN.md "Compiled runs"; 0 when it runs them interpreted: LDS
 * frames, metering, WB_JIT=0, or a compile failure, whose message WasmEdge_BatchGetLastError
 * then returns until the next error). Results never depend on it. */
WASMEDGE_BATCH_API uint32_t WasmEdge_BatchGetCompiledRuns(const WasmEdge_BatchContext *Cxt);

/* The execution engine the context runs, for reports (DESIGN.md "Execution engines"):
 * "<core>/<frames>", core one of "compiled-runs" (with "+simt" / "+trip" for the
 * scheduling inside them), "threaded-core" (the hand-written handlers, no compiled runs),
 * "compiled-step"; frames "vgpr-frames", "lds-frames" or "hbm-frames"; "+metered" when the
 * context meters gas. A context that wanted compiled runs and got none (a compile failure)
 * says "threaded-core (compiled runs failed)". Valid until the next call on the context;
 * "" for NULL. Results never depend on it. */
WASMEDGE_BATCH_API const char *WasmEdge_BatchGetEngine(const WasmEdge_BatchContext *Cxt);

/* The interleave granule in use, in bytes (WasmEdge_BatchConfigure::MemoryGranule).
 * Layout only: results never depend on it. */
WASMEDGE_BATCH_API uint32_t WasmEdge_BatchGetMemoryGranule(const WasmEdge_BatchContext *Cxt);

/* Pages of every instance's memory in the reserved layout, which every execution path
 * addresses directly (pages past it come from pool rows through a page table). It starts at
 * MemoryReservePages (or the module's choice) and, at a BatchReset after a run whose
 * instances grew past it, takes the largest memory they reached (within 3/4 of the device
 * memory, and MemoryPoolBytes past the initial layout). Layout only: results never depend
 * on it. */
WASMEDGE_BATCH_API uint32_t WasmEdge_BatchGetReservedPages(const WasmEdge_BatchContext *Cxt);
/* Pages every instance has reserved for memory MemIdx >= 1 (MultiMemories): memory.grow on
 * it returns -1 past them (0 for an index the module does not have). */
WASMEDGE_BATCH_API uint32_t WasmEdge_BatchGetExtraMemoryPages(const WasmEdge_BatchContext *Cxt,
                                                              uint32_t MemIdx);

/* Hash of every instance's final linear memory 0 (definition in DESIGN.md; the oracle
 * computes the same function). Hashes: [NumInstances]. */
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchMemoryHash(WasmEdge_BatchContext *Cxt,
                                                            uint64_t *Hashes);
/* Copy Len bytes of instance Inst's linear memory starting at Off into Dst
 * (MemoryOutOfBounds 0x88 if outside its current size). */
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchGetMemory(WasmEdge_BatchContext *Cxt,
                                                           uint32_t Inst, uint32_t Off,
                                                           uint8_t *Dst, uint32_t Len);
/* Write Len bytes into instance Inst's linear memory at Off (0x88 if outside it). */
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchSetMemory(WasmEdge_BatchContext *Cxt,
                                                           uint32_t Inst, uint32_t Off,
                                                           const uint8_t *Src, uint32_t Len);
/* Exported tables and globals of one instance, by export name (the batched form of
 * WasmEdge_StoreFindTable/FindGlobal + WasmEdge_TableInstanceGetData/SetData/GetSize,
 * lib/api/wasmedge.cpp:2099-2139, and WasmEdge_GlobalInstanceGetValue/SetValue,
 * :2273-2295). Inst = WASMEDGE_BATCH_ALL_INSTANCES writes every instance. Reference
 * values: a funcref is the module's function index; an externref is any 64-bit host value
 * (a pointer, as WasmEdge_ValueGenExternRef makes, wasmedge.h:254,318), given back
 * unchanged wherever it leaves the batch (results, host-function arguments, table and
 * global reads); null is 0xFFFFFFFF for both. (On the device refs are 32-bit: a value
 * from 2^31 up is carried as a handle the context interns.) TableGetData/SetData: TableOutOfBounds (0x87) past the instance's table
 * size, RefTypeMismatch (0x8E) for a value of the wrong reference type. GlobalSetValue
 * ignores a constant global or a value of another type, as the reference does. An
 * unknown export name gives FuncNotFound (0x05). Writes persist until BatchReset. */
#define WASMEDGE_BATCH_ALL_INSTANCES 0xFFFFFFFFu
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchTableGetSize(WasmEdge_BatchContext *Cxt,
                                                              const WasmEdge_String TableName,
                                                              uint32_t Inst, uint32_t *Size);
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchTableGetData(WasmEdge_BatchContext *Cxt,
                                                              const WasmEdge_String TableName,
                                                              uint32_t Inst, WasmEdge_Value *Data,
                                                              uint32_t Offset);
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchTableSetData(WasmEdge_BatchContext *Cxt,
                                                              const WasmEdge_String TableName,
                                                              uint32_t Inst, WasmEdge_Value Data,
                                                              uint32_t Offset);
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchGlobalGetValue(WasmEdge_BatchContext *Cxt,
                                                                const WasmEdge_String GlobalName,
                                                                uint32_t Inst, WasmEdge_Value *Value);
WASMEDGE_BATCH_API WasmEdge_Result WasmEdge_BatchGlobalSetValue(WasmEdge_BatchContext *Cxt,
                                                                const WasmEdge_String GlobalName,
                                                                uint32_t Inst, WasmEdge_Value Value);
/* Current page count of instance Inst's memory. */
WASMEDGE_BATCH_API uint32_t WasmEdge_BatchGetMemoryPages(WasmEdge_BatchContext *Cxt,
                                                         uint32_t Inst);
WASMEDGE_BATCH_API uint32_t WasmEdge_BatchGetInstanceCount(const WasmEdge_BatchContext *Cxt);
/* Hash of the sources this library was built from (wasmedge_amd/csrc/srchash.py): lets a
 * caller check that the library it loaded matches the checked-out tree (the batched form
 * of the reference's WasmEdge_VersionGet, wasmedge.h). */
WASMEDGE_BATCH_API const char *WasmEdge_BatchGetBuildHash(void);
/* Human-readable description of the last failure on this context (or of the last
 * failed BatchCreate when Cxt is NULL). */
WASMEDGE_BATCH_API const char *WasmEdge_BatchGetLastError(const WasmEdge_BatchContext *Cxt);
/* Number of device instructions and max wasm instructions folded into one dispatch. */
WASMEDGE_BATCH_API uint32_t WasmEdge_BatchGetCodeSize(const WasmEdge_BatchContext *Cxt);
WASMEDGE_BATCH_API void WasmEdge_BatchDelete(WasmEdge_BatchContext *Cxt);

#ifdef __cplusplus
}
#endif
#endif
