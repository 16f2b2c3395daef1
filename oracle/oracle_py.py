"""ctypes binding of the oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.om_load.restype = ctypes.c_void_p
        L.om_load.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                              ctypes.POINTER(ctypes.c_int)]
        L.om_free.argtypes = [ctypes.c_void_p]
        L.om_find_func.restype = ctypes.c_int
        L.om_find_func.argtypes = [ctypes.c_void_p, ctypes.c_char_p,
                                   ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p,
                                   ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p]
        L.om_instantiate.restype = ctypes.c_void_p
        L.om_instantiate.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.om_inst_free.argtypes = [ctypes.c_void_p]
        L.om_invoke.restype = ctypes.c_int
        L.om_invoke.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
        L.om_set_cost_limit.restype = None
        L.om_set_cost_limit.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.om_set_tail_call.restype = None
        L.om_set_tail_call.argtypes = [ctypes.c_int]
        L.om_set_multi_memory.restype = None
        L.om_set_multi_memory.argtypes = [ctypes.c_int]
        L.om_set_metering.restype = None
        L.om_set_metering.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
        L.om_cost_sum.restype = ctypes.c_uint64
        L.om_cost_sum.argtypes = [ctypes.c_void_p]
        L.om_terminated.restype = ctypes.c_int
        L.om_terminated.argtypes = [ctypes.c_void_p]
        L.om_mem_pages.restype = ctypes.c_uint32
        L.om_mem_pages.argtypes = [ctypes.c_void_p]
        L.om_mem_data.restype = ctypes.c_void_p
        L.om_mem_data.argtypes = [ctypes.c_void_p]
        L.om_mem_hash.restype = ctypes.c_uint64
        L.om_mem_hash.argtypes = [ctypes.c_void_p]
        L.om_hash_bytes.restype = ctypes.c_uint64
        L.om_hash_bytes.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]
        L.om_set_lazy_imports.restype = None
        L.om_set_lazy_imports.argtypes = [ctypes.c_int]
        L.om_set_host_cost.restype = None
        L.om_set_host_cost.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64]
        L.om_set_extern_value.restype = None
        L.om_set_extern_value.argtypes = [ctypes.c_uint32, ctypes.c_int32]
        L.om_table_set.restype = ctypes.c_int
        L.om_table_set.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.om_global_get.restype = None
        L.om_global_get.argtypes = [ctypes.c_void_p, ctypes.c_uint32,
                                    ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.om_run_batch.restype = ctypes.c_double
        L.om_run_batch.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.om_run_batch_mb.restype = ctypes.c_double
        L.om_run_batch_mb.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32] + \
            [ctypes.c_void_p] * 6 + [ctypes.c_int]
        L.om_run_batch_ms.restype = ctypes.c_double
        L.om_run_batch_ms.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32] + \
            [ctypes.c_void_p] * 7 + [ctypes.c_int]
        L.om_clear_imports.restype = None
        L.om_add_import.restype = None
        L.om_add_import.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_uint32] * 5 + \
            [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        cpp = ctypes.POINTER(ctypes.c_char_p)
        L.om_set_wasi.restype = None
        L.om_set_wasi.argtypes = [ctypes.c_int, cpp, ctypes.c_uint32, cpp, ctypes.c_uint32]
        L.om_set_wasi_preopens.restype = None
        L.om_set_wasi_preopens.argtypes = [cpp, ctypes.c_uint32]
        L.om_set_wasi_deterministic.restype = None
        L.om_set_wasi_deterministic.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        L.om_wasi_set_lane.restype = None
        L.om_wasi_set_lane.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.om_set_instance_args.restype = None
        L.om_set_instance_args.argtypes = [ctypes.c_void_p, cpp, ctypes.c_uint32]
        L.om_wasi_exit_code.restype = ctypes.c_uint32
        L.om_wasi_exit_code.argtypes = [ctypes.c_void_p]
        L.om_wasi_output.restype = ctypes.c_uint64
        L.om_wasi_output.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]
        _lib = L
    return _lib


# The reference ends a proc_exit'ed run "successfully" with unspecified return values
# (engine.cpp:62-64); the wrappers report it as this code with no values, like the
# batched path's PerInstance.
TERMINATED = 0x01


class OracleError(Exception):
    def __init__(self, code):
        super().__init__("oracle error 0x%02x" % code)
        self.code = code


def _split(v):
    v &= (1 << 128) - 1
    return v & 0xFFFFFFFFFFFFFFFF, v >> 64


class Module:
    """A loaded + validated module in the oracle (one per wasm binary)."""

    def __init__(self, wasm, page_limit=65536, tail_call=False, multi_memory=False):
        """tail_call: the TailCall proposal (return_call / return_call_indirect) is on;
        multi_memory: the MultiMemories proposal."""
        L = lib()
        err = ctypes.c_int(0)
        L.om_set_tail_call(1 if tail_call else 0)
        L.om_set_multi_memory(1 if multi_memory else 0)
        try:
            self._h = L.om_load(wasm, len(wasm), page_limit, ctypes.byref(err))
        finally:
            L.om_set_tail_call(0)
            L.om_set_multi_memory(0)
        if not self._h:
            raise OracleError(err.value)
        self.wasm = wasm

    def __del__(self):
        if getattr(self, "_h", None):
            lib().om_free(self._h)
            self._h = None

    def func(self, name):
        np_, nr = ctypes.c_uint32(), ctypes.c_uint32()
        pt, rt = ctypes.create_string_buffer(64), ctypes.create_string_buffer(64)
        idx = lib().om_find_func(self._h, name.encode(), ctypes.byref(np_), pt,
                                 ctypes.byref(nr), rt)
        if idx < 0:
            raise KeyError(name)
        return idx, list(pt.raw[:np_.value]), list(rt.raw[:nr.value])

    def run(self, name, args):
        """Fresh instance, invoke, return (code, results(int list), count, memhash)."""
        L = lib()
        idx, pt, rt = self.func(name)
        err = ctypes.c_int(0)
        inst = L.om_instantiate(self._h, ctypes.byref(err))
        if not inst:
            return err.value, [], 0, 0
        try:
            params = (ctypes.c_uint64 * (2 * max(1, len(pt))))()
            for k, a in enumerate(args):
                params[2 * k], params[2 * k + 1] = _split(a)
            res = (ctypes.c_uint64 * (2 * max(1, len(rt))))()
            cnt = ctypes.c_uint64(0)
            code = L.om_invoke(inst, idx, params, res, ctypes.byref(cnt))
            if code == 0 and L.om_terminated(inst):
                code = TERMINATED
            vals = [res[2 * k] | (res[2 * k + 1] << 64) for k in range(len(rt))] if code == 0 else []
            return code, vals, cnt.value, L.om_mem_hash(inst)
        finally:
            L.om_inst_free(inst)

    def run_with_memory(self, name, args):
        L = lib()
        idx, pt, rt = self.func(name)
        err = ctypes.c_int(0)
        inst = L.om_instantiate(self._h, ctypes.byref(err))
        if not inst:
            return err.value, [], 0, b""
        try:
            params = (ctypes.c_uint64 * (2 * max(1, len(pt))))()
            for k, a in enumerate(args):
                params[2 * k], params[2 * k + 1] = _split(a)
            res = (ctypes.c_uint64 * (2 * max(1, len(rt))))()
            cnt = ctypes.c_uint64(0)
            code = L.om_invoke(inst, idx, params, res, ctypes.byref(cnt))
            vals = [res[2 * k] | (res[2 * k + 1] << 64) for k in range(len(rt))] if code == 0 else []
            n = L.om_mem_pages(inst) * 65536
            mem = ctypes.string_at(L.om_mem_data(inst), n) if n else b""
            return code, vals, cnt.value, mem
        finally:
            L.om_inst_free(inst)

    def run_batch(self, name, params_u64, n, threads=1):
        """params_u64: numpy uint64 array shape [n, nparams, 2]. Returns dict of arrays."""
        import numpy as np
        L = lib()
        idx, pt, rt = self.func(name)
        params = np.ascontiguousarray(params_u64, dtype=np.uint64).reshape(n, len(pt), 2)
        results = np.zeros((n, max(1, len(rt)), 2), dtype=np.uint64)
        codes = np.zeros(n, dtype=np.uint8)
        counts = np.zeros(n, dtype=np.uint64)
        hashes = np.zeros(n, dtype=np.uint64)
        mem_bytes = np.zeros(n, dtype=np.uint64)
        store_bytes = np.zeros(n, dtype=np.uint64)
        secs = L.om_run_batch_ms(self._h, idx, n, params.ctypes.data, results.ctypes.data,
                                 codes.ctypes.data, counts.ctypes.data, hashes.ctypes.data,
                                 mem_bytes.ctypes.data, store_bytes.ctypes.data, threads)
        return {"results": results[:, :len(rt), :], "codes": codes, "counts": counts,
                "hashes": hashes, "mem_bytes": mem_bytes, "store_bytes": store_bytes,
                "seconds": secs}


class Instance:
    """One instantiated module (om_instantiate, start function included) that keeps its
    state -- memory, globals, tables -- across invoke() calls, like a module
    instantiated once in the reference VM and executed repeatedly."""

    def __init__(self, module, cost_limit=0, cost_table=None):
        """cost_limit / cost_table: gas metering from instantiation on (the constant
        expressions and the start function spend gas too); cost_table = a list of costs
        by OpCode (missing entries 0), None = unit costs."""
        L = lib()
        self.module = module
        err = ctypes.c_int(0)
        tab = None
        if cost_table is not None:
            tab = (ctypes.c_uint64 * max(1, len(cost_table)))(*cost_table)
        L.om_set_metering(cost_limit, tab, len(cost_table) if cost_table is not None else 0)
        try:
            self._h = L.om_instantiate(module._h, ctypes.byref(err))
        finally:
            L.om_set_metering(0, None, 0)
        self.error = err.value if not self._h else 0

    def cost_sum(self):
        return lib().om_cost_sum(self._h) if self._h else 0

    def __del__(self):
        if getattr(self, "_h", None):
            lib().om_inst_free(self._h)
            self._h = None

    def invoke(self, name, args):
        """(code, results, count, memhash) of one invocation on this instance."""
        if not self._h:
            return self.error, [], 0, 0
        L = lib()
        idx, pt, rt = self.module.func(name)
        params = (ctypes.c_uint64 * (2 * max(1, len(pt))))()
        for k, a in enumerate(args):
            params[2 * k], params[2 * k + 1] = _split(a)
        res = (ctypes.c_uint64 * (2 * max(1, len(rt))))()
        cnt = ctypes.c_uint64(0)
        code = L.om_invoke(self._h, idx, params, res, ctypes.byref(cnt))
        if code == 0 and L.om_terminated(self._h):
            code = TERMINATED
        vals = [res[2 * k] | (res[2 * k + 1] << 64) for k in range(len(rt))] if code == 0 else []
        return code, vals, cnt.value, L.om_mem_hash(self._h)


    def wasi_output(self, fd=1):
        p = ctypes.c_void_p()
        n = lib().om_wasi_output(self._h, fd, ctypes.byref(p))
        return ctypes.string_at(p.value, n) if n else b""

    def wasi_exit_code(self):
        return lib().om_wasi_exit_code(self._h)

    def memory(self, off, n):
        """n bytes of linear memory 0 from off."""
        L = lib()
        assert off + n <= L.om_mem_pages(self._h) * 65536
        return ctypes.string_at(L.om_mem_data(self._h) + off, n)

    def set_lane(self, lane):
        """The instance id its WASI generator is keyed on (fd numbers, random_get)."""
        lib().om_wasi_set_lane(self._h, lane)

    def set_args(self, args):
        """This instance's own WASI command line (one Environ per VM)."""
        a = (ctypes.c_char_p * max(len(args), 1))(*[x.encode() for x in args])
        lib().om_set_instance_args(self._h, a, len(args))

    def table_set(self, tab, off, ref):
        """Write one table entry (ref: function index / externref handle, None = null);
        returns the ErrCode (0x87 out of bounds)."""
        return lib().om_table_set(self._h, tab, off, (1 << 64) - 1 if ref is None else ref)

    def global_get(self, g):
        lo, hi = ctypes.c_uint64(0), ctypes.c_uint64(0)
        lib().om_global_get(self._h, g, ctypes.byref(lo), ctypes.byref(hi))
        return lo.value | (hi.value << 64)


def set_lazy_imports(on):
    """Instantiate modules with imports no test host module provides (calls fail)."""
    lib().om_set_lazy_imports(1 if on else 0)


def set_wasi(on, args=(), envs=(), preopens=(), deterministic=None):
    """Bind the WASI subset (wasi_snapshot_preview1) for later instantiations, with these
    args/envs shared by every instance (the batched path's WasmEdge_BatchInitWASI) and
    these preopened directories (fds 3, 4, ...); deterministic: (seed, clock_ns) as
    WasmEdge_BatchWASISetDeterministic."""
    def arr(v):
        return (ctypes.c_char_p * max(len(v), 1))(*[x.encode() for x in v])
    lib().om_set_wasi(1 if on else 0, arr(list(args)), len(args), arr(list(envs)), len(envs))
    lib().om_set_wasi_preopens(arr(list(preopens)), len(preopens))
    seed, clock = deterministic or (0, 0)
    lib().om_set_wasi_deterministic(1 if deterministic else 0, seed, clock)


def set_imports(imports):
    """Provided tables / memories / globals for modules loaded afterwards: dicts with
    module, name, kind (1 table, 2 memory, 3 global), type, mut, min, max (None = no max),
    value (global)."""
    L = lib()
    L.om_clear_imports()
    for i in imports or []:
        v = int(i.get("value", 0)) & ((1 << 128) - 1)
        mx = i.get("max")
        L.om_add_import(i["module"].encode(), i["name"].encode(), i["kind"], i.get("type", 0),
                        1 if i.get("mut") else 0, i.get("min", 0), mx or 0, 0 if mx is None else 1,
                        v & ((1 << 64) - 1), v >> 64)


def set_host_costs(costs):
    """Costs of the test host functions, {(module, name): cost} (HostFunctionBase::Cost);
    charged under metering before the function runs (helper.cpp:59-64). {} clears them."""
    L = lib()
    L.om_set_host_cost(None, None, 0)
    for (mod, name), c in (costs or {}).items():
        L.om_set_host_cost(mod.encode(), name.encode(), int(c))


def set_extern_value(handle, value):
    """The int32 an externref handle points to, for the "extern" test host module."""
    lib().om_set_extern_value(handle, value)


def hash_bytes(data, pages):
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    return lib().om_hash_bytes(buf, len(data), pages)
