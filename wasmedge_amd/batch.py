"""Python host mirror of the batched C ABI (include/wasmedge_batch.h) over ctypes.

Mirrors the reference VM/C-API flow (lib/vm/vm.cpp, include/api/wasmedge/wasmedge.h):
load -> validate -> instantiate -> execute, but for N instances at once.  The product
path is the HIP library `libwasmedge_batch.so`; there is no CPU fallback -- if the library
or a GPU is missing, construction raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# WB_BATCH_LIB selects a profiling variant (libwasmedge_batch_stats.so, tools/ only)
LIB_PATH = os.environ.get("WB_BATCH_LIB") or os.path.join(_HERE, "libwasmedge_batch.so")

# valtypes (include/api/wasmedge/enum_types.h)
I32, I64, F32, F64, V128, FUNCREF, EXTERNREF = 0x7F, 0x7E, 0x7D, 0x7C, 0x7B, 0x70, 0x6F

# WasmEdge_Value: {uint128_t Value; enum WasmEdge_ValType Type;} -> 32 bytes (16-aligned)
VALUE_DTYPE = np.dtype([("lo", "<u8"), ("hi", "<u8"), ("type", "<u4"), ("pad", "<u4", (3,))])

# per-instance status codes (reference ErrCodes, include/common/enum.inc:717-745)
STATUS_NAMES = {0x00: "ok", 0x07: "interrupted", 0x84: "integer divide by zero",
                0x85: "integer overflow", 0x86: "invalid conversion to integer",
                0x87: "out of bounds table access", 0x88: "out of bounds memory access",
                0x89: "unreachable", 0x8A: "uninitialized element", 0x8B: "undefined element",
                0x8C: "indirect call type mismatch", 0xB0: "call stack exhausted",
                0xB1: "host call (yield path not implemented)"}


ALL_INSTANCES = 0xFFFFFFFF
REF_NULL = 0xFFFFFFFF   # null funcref / externref on the device (32-bit references)


class _Value(ctypes.Structure):
    """WasmEdge_Value passed by value: uint128 as two u64 words, then the type."""
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64), ("type", ctypes.c_uint32),
                ("pad", ctypes.c_uint32 * 3)]

    @classmethod
    def make(cls, value, vtype):
        v = int(value) & ((1 << 128) - 1)
        return cls(v & 0xFFFFFFFFFFFFFFFF, v >> 64, vtype)

    def int(self):
        return self.lo | (self.hi << 64)


class WasmEdgeError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__("WasmEdge_Result 0x%02x %s" % (code, msg))
        self.code = code


class _Conf(ctypes.Structure):
    _fields_ = [("MaxMemoryPage", ctypes.c_uint32), ("CallStackCells", ctypes.c_uint32),
                ("MaxSteps", ctypes.c_uint64), ("TimeLimitSeconds", ctypes.c_double),
                ("DeviceOrdinal", ctypes.c_int32), ("CostLimit", ctypes.c_uint64),
                ("HostThreads", ctypes.c_uint32), ("CostTable", ctypes.c_void_p),
                ("CostTableLen", ctypes.c_uint32), ("MemoryGranule", ctypes.c_uint32),
                ("TailCall", ctypes.c_uint32), ("MemoryReservePages", ctypes.c_uint32),
                ("MemoryPoolBytes", ctypes.c_uint64), ("Devices", ctypes.POINTER(ctypes.c_int32)),
                ("DeviceCount", ctypes.c_uint32), ("Partition", ctypes.c_uint32),
                ("MultiMemories", ctypes.c_uint32), ("ExtraMemoryReservePages", ctypes.c_uint32),
                ("CallStackMaxBytes", ctypes.c_uint64)]

PARTITION_BLOCKS, PARTITION_INTERLEAVE = 0, 1


def placement(n, device_count, partition, inst):
    """(shard, lane) of instance `inst` in an n-instance batch over device_count devices
    (WasmEdge_BatchPlacement; no device needed)."""
    g, l = ctypes.c_uint32(), ctypes.c_uint32()
    r = lib().WasmEdge_BatchPlacement(n, device_count, partition, inst, ctypes.byref(g), ctypes.byref(l))
    if r.Code:
        raise WasmEdgeError(r.Code, "placement")
    return g.value, l.value


class _String(ctypes.Structure):
    _fields_ = [("Length", ctypes.c_uint32), ("Buf", ctypes.c_char_p)]


class _Import(ctypes.Structure):
    """WasmEdge_BatchImport: a provided table / memory / global."""
    _fields_ = [("ModuleName", _String), ("ExternalName", _String), ("Kind", ctypes.c_uint32),
                ("Min", ctypes.c_uint32), ("Max", ctypes.c_uint32), ("HasMax", ctypes.c_uint32),
                ("Type", ctypes.c_uint32), ("Mutable", ctypes.c_uint32),
                ("_align", ctypes.c_uint32 * 2),   # WasmEdge_Value is 16-byte aligned (uint128)
                ("Value", _Value)]


class _Result(ctypes.Structure):
    _fields_ = [("Code", ctypes.c_uint8)]


_lib = None

# WasmEdge_BatchHostFunc_t: WasmEdge_Result(void *Data, MemCxt *, const Value *, Value *).
# WasmEdge_Result is a one-byte struct, returned in a register exactly like a uint8_t.
HOST_FUNC = ctypes.CFUNCTYPE(ctypes.c_uint8, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p)


class HostMemory:
    """The calling instance's linear memory inside a host function
    (WasmEdge_BatchMemoryGetData / SetData)."""

    def __init__(self, handle):
        self._h = handle
        self.instance = lib().WasmEdge_BatchMemoryGetInstance(handle)

    def read(self, off, length):
        buf = ctypes.create_string_buffer(max(length, 1))
        r = lib().WasmEdge_BatchMemoryGetData(self._h, buf, off, length)
        if r.Code:
            raise WasmEdgeError(r.Code, "memory read")
        return buf.raw[:length]

    def write(self, off, data):
        r = lib().WasmEdge_BatchMemorySetData(self._h, bytes(data), off, len(data))
        if r.Code:
            raise WasmEdgeError(r.Code, "memory write")


def lib():
    """Load the HIP library (raises if it was not built -- no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError("libwasmedge_batch.so not built: run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
        L.WasmEdge_BatchCreate.restype = vp
        L.WasmEdge_BatchCreate.argtypes = [ctypes.POINTER(_Conf), ctypes.c_char_p, u32, u32,
                                           ctypes.POINTER(_Result)]
        L.WasmEdge_BatchCreateWithImports.restype = vp
        L.WasmEdge_BatchCreateWithImports.argtypes = [ctypes.POINTER(_Conf), ctypes.c_char_p, u32, u32,
                                                      ctypes.POINTER(_Import), u32,
                                                      ctypes.POINTER(_Result)]
        for name, args in [
            ("WasmEdge_BatchExecute", [vp, _String, vp, u32, vp, u32, vp, vp]),
            ("WasmEdge_BatchSetArgs", [vp, _String, vp, u32]),
            ("WasmEdge_BatchReset", [vp, ctypes.POINTER(ctypes.c_double)]),
            ("WasmEdge_BatchRun", [vp, ctypes.POINTER(ctypes.c_double)]),
            ("WasmEdge_BatchResults", [vp, vp, u32, vp, vp]),
            ("WasmEdge_BatchMemoryHash", [vp, vp]),
            ("WasmEdge_BatchGetMemory", [vp, u32, u32, vp, u32]),
        ]:
            f = getattr(L, name)
            f.restype = _Result
            f.argtypes = args
        L.WasmEdge_BatchGetMemoryPages.restype = u32
        L.WasmEdge_BatchGetMemoryPages.argtypes = [vp, u32]
        L.WasmEdge_BatchGetInstanceCount.restype = u32
        L.WasmEdge_BatchGetInstanceCount.argtypes = [vp]
        L.WasmEdge_BatchGetCodeSize.restype = u32
        L.WasmEdge_BatchGetCodeSize.argtypes = [vp]
        L.WasmEdge_BatchGetLastError.restype = ctypes.c_char_p
        L.WasmEdge_BatchGetLastError.argtypes = [vp]
        L.WasmEdge_BatchDelete.restype = None
        L.WasmEdge_BatchDelete.argtypes = [vp]
        for name, args in [
            ("WasmEdge_BatchSetMemory", [vp, u32, u32, ctypes.c_char_p, u32]),
            ("WasmEdge_BatchAddHostFunction", [vp, _String, _String, HOST_FUNC, vp]),
            ("WasmEdge_BatchAddHostFunctionWithCost", [vp, _String, _String, HOST_FUNC, vp, u64]),
            ("WasmEdge_BatchMemoryGetData", [vp, vp, u32, u32]),
            ("WasmEdge_BatchMemorySetData", [vp, ctypes.c_char_p, u32, u32]),
        ]:
            f = getattr(L, name)
            f.restype = _Result
            f.argtypes = args
        for name, args in [
            ("WasmEdge_BatchTableGetSize", [vp, _String, u32, ctypes.POINTER(u32)]),
            ("WasmEdge_BatchTableGetData", [vp, _String, u32, ctypes.POINTER(_Value), u32]),
            ("WasmEdge_BatchTableSetData", [vp, _String, u32, _Value, u32]),
            ("WasmEdge_BatchGlobalGetValue", [vp, _String, u32, ctypes.POINTER(_Value)]),
            ("WasmEdge_BatchGlobalSetValue", [vp, _String, u32, _Value]),
        ]:
            f = getattr(L, name)
            f.restype = _Result
            f.argtypes = args
        L.WasmEdge_BatchPlacement.restype = _Result
        L.WasmEdge_BatchPlacement.argtypes = [u32, u32, u32, u32, ctypes.POINTER(u32), ctypes.POINTER(u32)]
        L.WasmEdge_BatchInterrupt.restype = None
        L.WasmEdge_BatchInterrupt.argtypes = [vp]
        L.WasmEdge_BatchMemoryGetInstance.restype = u32
        L.WasmEdge_BatchMemoryGetInstance.argtypes = [vp]
        cpp = ctypes.POINTER(ctypes.c_char_p)
        L.WasmEdge_BatchGetTotalCosts.restype = _Result
        L.WasmEdge_BatchGetTotalCosts.argtypes = [vp, vp]
        L.WasmEdge_BatchInitWASI.restype = _Result
        L.WasmEdge_BatchInitWASI.argtypes = [vp, cpp, u32, cpp, u32]
        L.WasmEdge_BatchInitWASIWithPreopens.restype = _Result
        L.WasmEdge_BatchInitWASIWithPreopens.argtypes = [vp, cpp, u32, cpp, u32, cpp, u32]
        L.WasmEdge_BatchWASISetDeterministic.restype = _Result
        L.WasmEdge_BatchWASISetDeterministic.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64]
        L.WasmEdge_BatchWASISetInstanceArgs.restype = _Result
        L.WasmEdge_BatchWASISetInstanceArgs.argtypes = [vp, u32, cpp, u32]
        L.WasmEdge_BatchWASIGetExitCode.restype = u32
        L.WasmEdge_BatchWASIGetExitCode.argtypes = [vp, u32]
        L.WasmEdge_BatchWASIGetOutput.restype = u32
        L.WasmEdge_BatchWASIGetOutput.argtypes = [vp, u32, u32, vp, u32]
        L.WasmEdge_BatchGetCompiledRuns.restype = u32
        L.WasmEdge_BatchGetCompiledRuns.argtypes = [vp]
        L.WasmEdge_BatchGetMemoryGranule.restype = u32
        L.WasmEdge_BatchGetMemoryGranule.argtypes = [vp]
        L.WasmEdge_BatchGetReservedPages.restype = u32
        L.WasmEdge_BatchGetReservedPages.argtypes = [vp]
        L.WasmEdge_BatchGetExtraMemoryPages.restype = u32
        L.WasmEdge_BatchGetExtraMemoryPages.argtypes = [vp, u32]
        L.WasmEdge_BatchGetEngine.restype = ctypes.c_char_p
        L.WasmEdge_BatchGetEngine.argtypes = [vp]
        _lib = L
    return _lib


def make_values(rows, types):
    """rows: iterable of per-instance argument tuples (python ints, bit patterns for
    floats) or a numpy integer array [n, nparams]; types: list of valtypes."""
    if isinstance(rows, np.ndarray):
        arr = rows.reshape(rows.shape[0], -1)
        n = arr.shape[0]
        out = np.zeros((n, len(types)), VALUE_DTYPE)
        for k, t in enumerate(types):
            col = arr[:, k].astype(np.uint64) if arr.dtype.kind == "u" else \
                arr[:, k].astype(np.int64).view(np.uint64)
            if t in (I32, F32, FUNCREF):   # (an externref is any 64-bit host value)
                col = col & np.uint64(0xFFFFFFFF)
            out["lo"][:, k] = col
            out["type"][:, k] = t
        return out
    rows = list(rows)
    out = np.zeros((len(rows), len(types)), VALUE_DTYPE)
    for i, r in enumerate(rows):
        for k, t in enumerate(types):
            v = int(r[k]) & ((1 << 128) - 1)
            if t in (I32, F32, FUNCREF):
                v &= 0xFFFFFFFF
            elif t in (I64, F64, EXTERNREF):
                v &= (1 << 64) - 1
            out["lo"][i, k] = v & 0xFFFFFFFFFFFFFFFF
            out["hi"][i, k] = v >> 64
            out["type"][i, k] = t
    return out


class BatchContext:
    """N instances of one module on one GPU (WasmEdge_BatchContext)."""

    def __init__(self, wasm, n, max_memory_page=0, call_stack_cells=0, max_steps=0,
                 time_limit=0.0, device=-1, cost_limit=0, host_threads=0, cost_table=None,
                 memory_granule=0, imports=None, tail_call=False, memory_reserve_pages=0,
                 memory_pool_bytes=0, devices=None, partition=PARTITION_BLOCKS, multi_memory=False,
                 extra_memory_reserve_pages=0, call_stack_max_bytes=0):
        """cost_table: gas cost per OpCode (list; missing entries 0), None = unit costs;
        metering is on when cost_limit > 0. max_memory_page 0 = the reference's default
        page limit (65536); memory_reserve_pages / memory_pool_bytes: the device layout of
        grown memory (WasmEdge_BatchConfigure). devices: a list of HIP ordinals (repeats
        allowed) to spread the instances over from this process, by `partition`."""
        L = lib()
        tab = None
        if cost_table is not None:
            tab = np.ascontiguousarray(cost_table, np.uint64)
        conf = _Conf(max_memory_page, call_stack_cells, max_steps, time_limit, device, cost_limit,
                     host_threads, tab.ctypes.data if tab is not None and len(tab) else None,
                     len(tab) if tab is not None else 0, memory_granule, 1 if tail_call else 0,
                     memory_reserve_pages, memory_pool_bytes)
        conf.MultiMemories = 1 if multi_memory else 0
        conf.ExtraMemoryReservePages = extra_memory_reserve_pages
        conf.CallStackMaxBytes = call_stack_max_bytes
        if devices is not None and len(devices) == 1:
            conf.DeviceOrdinal = devices[0]
        if devices is not None and len(devices) > 1:
            self._devices = (ctypes.c_int32 * len(devices))(*devices)
            conf.Devices = self._devices
            conf.DeviceCount = len(devices)
            conf.Partition = partition
        res = _Result(0)
        imps = imports or []
        arr = (_Import * max(1, len(imps)))()
        self._import_names = []
        for k, i in enumerate(imps):
            mod, nm = i["module"].encode(), i["name"].encode()
            self._import_names += [mod, nm]
            mx = i.get("max")
            arr[k] = _Import(_String(len(mod), mod), _String(len(nm), nm), i["kind"], i.get("min", 0),
                             mx or 0, 0 if mx is None else 1, i.get("type", 0),
                             1 if i.get("mut") else 0, (ctypes.c_uint32 * 2)(),
                             _Value.make(i.get("value", 0), i.get("type", 0)))
        self._h = L.WasmEdge_BatchCreateWithImports(ctypes.byref(conf), bytes(wasm), len(wasm), n,
                                                    arr, len(imps), ctypes.byref(res))
        if not self._h:
            raise WasmEdgeError(res.Code, L.WasmEdge_BatchGetLastError(None).decode())
        self.n = n
        self.func = None

    def close(self):
        if getattr(self, "_h", None):
            lib().WasmEdge_BatchDelete(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def _check(self, r):
        if r.Code:
            raise WasmEdgeError(r.Code, lib().WasmEdge_BatchGetLastError(self._h).decode())

    @staticmethod
    def _name(func):
        b = func.encode()
        return _String(len(b), b)

    def set_args(self, func, values):
        values = np.ascontiguousarray(values, VALUE_DTYPE)
        # WasmEdge_BatchSetArgs reads NumInstances rows: a shorter array would be read past
        if values.ndim != 2 or values.shape[0] != self.n:
            raise ValueError("values must be [%d instances][params], got shape %s"
                             % (self.n, values.shape))
        nparams = values.shape[1]
        self._check(lib().WasmEdge_BatchSetArgs(self._h, self._name(func),
                                                values.ctypes.data if values.size else None,
                                                nparams))
        self.func = func
        self._keep = values

    def reset(self, timed=True):
        """Re-instantiate every instance; returns the reset kernels' time (timed=False: no
        host synchronisation, returns 0 -- the next run orders after it on the stream)."""
        t = ctypes.c_double(0)
        self._check(lib().WasmEdge_BatchReset(self._h, ctypes.byref(t) if timed else None))
        return t.value

    def run(self):
        t = ctypes.c_double(0)
        self._check(lib().WasmEdge_BatchRun(self._h, ctypes.byref(t)))
        return t.value

    def results(self, nret):
        rets = np.zeros((self.n, max(nret, 1)), VALUE_DTYPE)
        status = np.zeros(self.n, np.uint8)
        counts = np.zeros(self.n, np.uint64)
        self._check(lib().WasmEdge_BatchResults(self._h, rets.ctypes.data, nret,
                                                status.ctypes.data, counts.ctypes.data))
        return rets[:, :nret], status, counts

    def execute(self, func, values, nret):
        """Invoke `func` on every instance (WasmEdge_BatchExecute: state persists from
        the previous invocation; reset() re-instantiates). Returns (returns[n, nret]
        VALUE_DTYPE, status, counts)."""
        self.set_args(func, values)
        self.run()
        return self.results(nret)

    def total_costs(self):
        """Each instance's gas total (WasmEdge_BatchGetTotalCosts)."""
        c = np.zeros(self.n, np.uint64)
        self._check(lib().WasmEdge_BatchGetTotalCosts(self._h, c.ctypes.data))
        return c

    def memory_hash(self):
        h = np.zeros(self.n, np.uint64)
        self._check(lib().WasmEdge_BatchMemoryHash(self._h, h.ctypes.data))
        return h

    def memory(self, inst, off, length):
        buf = ctypes.create_string_buffer(length)
        self._check(lib().WasmEdge_BatchGetMemory(self._h, inst, off, buf, length))
        return buf.raw

    def memory_pages(self, inst):
        return lib().WasmEdge_BatchGetMemoryPages(self._h, inst)

    def code_size(self):
        return lib().WasmEdge_BatchGetCodeSize(self._h)

    def compiled_runs(self):
        """Straight-line runs compiled for the V-frame core (WasmEdge_BatchGetCompiledRuns)."""
        return lib().WasmEdge_BatchGetCompiledRuns(self._h)

    def memory_granule(self):
        """The interleave granule in use, bytes (WasmEdge_BatchGetMemoryGranule)."""
        return lib().WasmEdge_BatchGetMemoryGranule(self._h)

    def reserved_pages(self):
        """Pages of every instance in the directly addressed layout
        (WasmEdge_BatchGetReservedPages)."""
        return lib().WasmEdge_BatchGetReservedPages(self._h)

    def extra_memory_pages(self, mem):
        """Pages reserved per instance for memory `mem` >= 1 (WasmEdge_BatchGetExtraMemoryPages)."""
        return lib().WasmEdge_BatchGetExtraMemoryPages(self._h, mem)

    def engine(self):
        """The execution engine the context runs, e.g. "compiled-runs+simt/vgpr-frames"
        (WasmEdge_BatchGetEngine)."""
        return lib().WasmEdge_BatchGetEngine(self._h).decode()

    def interrupt(self):
        lib().WasmEdge_BatchInterrupt(self._h)

    def set_memory(self, inst, off, data):
        self._check(lib().WasmEdge_BatchSetMemory(self._h, inst, off, bytes(data), len(data)))

    # exported tables / globals of one instance (WasmEdge_TableInstance*/GlobalInstance*);
    # inst=None writes every instance
    def table_size(self, name, inst):
        n = ctypes.c_uint32(0)
        self._check(lib().WasmEdge_BatchTableGetSize(self._h, self._name(name), inst, ctypes.byref(n)))
        return n.value

    def table_get(self, name, inst, off):
        v = _Value()
        self._check(lib().WasmEdge_BatchTableGetData(self._h, self._name(name), inst, ctypes.byref(v), off))
        return v.int(), v.type

    def table_set(self, name, inst, off, value, vtype):
        inst = ALL_INSTANCES if inst is None else inst
        self._check(lib().WasmEdge_BatchTableSetData(self._h, self._name(name), inst,
                                                     _Value.make(value, vtype), off))

    def global_get(self, name, inst):
        v = _Value()
        self._check(lib().WasmEdge_BatchGlobalGetValue(self._h, self._name(name), inst, ctypes.byref(v)))
        return v.int(), v.type

    def global_set(self, name, inst, value, vtype):
        inst = ALL_INSTANCES if inst is None else inst
        self._check(lib().WasmEdge_BatchGlobalSetValue(self._h, self._name(name), inst,
                                                       _Value.make(value, vtype)))

    def add_host_function(self, module, name, fn, nparams, nresults, cost=0):
        """Bind `fn(mem: HostMemory, args: list[int]) -> (code, results: list[int])` to
        the import module.name (WasmEdge_BatchAddHostFunction; with a gas `cost`,
        WasmEdge_BatchAddHostFunctionWithCost). Values are raw bits (uint128 as python
        ints); code 0 = success, else the ErrCode ending the instance (0x01 Terminated)."""
        def tramp(_data, memcxt, params, returns):
            pv = np.ctypeslib.as_array((ctypes.c_uint8 * (32 * max(nparams, 1))).from_address(params)) \
                if nparams else None
            args = []
            if nparams:
                vals = pv.view(VALUE_DTYPE)
                args = [int(vals["lo"][k]) | (int(vals["hi"][k]) << 64) for k in range(nparams)]
            try:
                code, res = fn(HostMemory(memcxt), args)
            except WasmEdgeError as e:
                return e.code
            if code == 0 and nresults:
                rv = np.ctypeslib.as_array((ctypes.c_uint8 * (32 * nresults)).from_address(returns)).view(VALUE_DTYPE)
                for k in range(nresults):
                    v = int(res[k]) & ((1 << 128) - 1)
                    rv["lo"][k] = v & 0xFFFFFFFFFFFFFFFF
                    rv["hi"][k] = v >> 64
            return code
        cb = HOST_FUNC(tramp)
        self._hosts = getattr(self, "_hosts", []) + [cb]   # keep the trampoline alive
        self._check(lib().WasmEdge_BatchAddHostFunctionWithCost(self._h, self._name(module),
                                                                self._name(name), cb, None, cost))


    # built-in WASI subset (WasmEdge_BatchInitWASIWithPreopens): args/envs shared by every
    # instance, preopened directories as fds 3, 4, ...
    def init_wasi(self, args=(), envs=(), preopens=()):
        a, e, p = _cstrs(args), _cstrs(envs), _cstrs(preopens)
        self._check(lib().WasmEdge_BatchInitWASIWithPreopens(self._h, a, len(args), e, len(envs),
                                                             p, len(preopens)))

    def wasi_deterministic(self, seed, clock_ns):
        """Reproducible fd numbers / random_get / clocks (WasmEdge_BatchWASISetDeterministic)."""
        self._check(lib().WasmEdge_BatchWASISetDeterministic(self._h, seed, clock_ns))

    def set_instance_args(self, inst, args):
        """Instance `inst`'s own command line (WasmEdge_BatchWASISetInstanceArgs)."""
        self._check(lib().WasmEdge_BatchWASISetInstanceArgs(self._h, inst, _cstrs(args), len(args)))

    def wasi_exit_code(self, inst):
        return lib().WasmEdge_BatchWASIGetExitCode(self._h, inst)

    def wasi_output(self, inst, fd=1):
        n = lib().WasmEdge_BatchWASIGetOutput(self._h, inst, fd, None, 0)
        buf = ctypes.create_string_buffer(max(n, 1))
        lib().WasmEdge_BatchWASIGetOutput(self._h, inst, fd, buf, n)
        return buf.raw[:n]


def _cstrs(v):
    v = list(v)
    return (ctypes.c_char_p * max(len(v), 1))(*[x.encode() for x in v])


def ret_ints(rets):
    """Return values (VALUE_DTYPE array) as python ints (uint128)."""
    lo = rets["lo"].astype(object)
    hi = rets["hi"].astype(object)
    return lo + hi * (1 << 64)
