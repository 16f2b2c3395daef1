"""The test host module "env" on the batched path: the same functions the oracle defines
(oracle/wasm_oracle_exec.inc host_call), registered through WasmEdge_BatchAddHostFunction.
Used by the host-import yield-path parity tests."""
import struct

from wasmedge_amd.batch import WasmEdgeError

MEM_OOB, HOST_FAILED, TERMINATED = 0x88, 0x8D, 0x01
M64 = (1 << 64) - 1


def _f64(bits):
    return struct.unpack("<d", struct.pack("<Q", bits & M64))[0]


def _bits(d):
    return struct.unpack("<Q", struct.pack("<d", d))[0]


def _i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >> 31 else v


def add_i64(mem, a):
    return 0, [(a[0] + a[1]) & M64]


def mem_sum(mem, a):
    p, n = a[0] & 0xFFFFFFFF, a[1] & 0xFFFFFFFF
    try:
        return 0, [sum(mem.read(p, n)) & 0xFFFFFFFF]
    except WasmEdgeError:
        return MEM_OOB, []


def mem_fill(mem, a):
    p, n, b = a[0] & 0xFFFFFFFF, a[1] & 0xFFFFFFFF, a[2] & 0xFF
    try:
        mem.write(p, bytes([b]) * n)
    except WasmEdgeError:
        return MEM_OOB, []
    return 0, []


def fail(mem, a):
    return (HOST_FAILED, []) if a[0] & 0xFFFFFFFF else (0, [7])


def exit_(mem, a):
    return TERMINATED, []


def mix(mem, a):
    return 0, [_bits(float(_i32(a[0])) * _f64(a[1]) + 0.5)]


ENV = {"add_i64": (add_i64, 2, 1), "mem_sum": (mem_sum, 2, 1), "mem_fill": (mem_fill, 3, 0),
       "fail": (fail, 1, 1), "exit": (exit_, 1, 0), "mix": (mix, 2, 1)}


# ---- the reference API test's import module "extern" (test/api/APIUnitTest.cpp:48-95):
# {externref, i32} -> {i32} over the int32 an externref points to. Here an externref is a
# 32-bit handle; EXTERN_VALUES maps it to its int32 (oracle: om_set_extern_value).
EXTERN_VALUES = {}


def _extern_op(op):
    def f(mem, a):
        h = a[0] & 0xFFFFFFFF
        if h >= 256 or h not in EXTERN_VALUES:
            return HOST_FAILED, []
        x, y = EXTERN_VALUES[h], _i32(a[1])
        if op == "div":
            if y == 0 or (x == -(1 << 31) and y == -1):
                return HOST_FAILED, []
            q = abs(x) // abs(y)
            v = -q if (x < 0) != (y < 0) else q
        else:
            v = {"add": x + y, "sub": x - y, "mul": x * y}[op]
        return 0, [v & 0xFFFFFFFF]
    return f


EXTERN = {"func-add": (_extern_op("add"), 2, 1), "func-sub": (_extern_op("sub"), 2, 1),
          "func-mul": (_extern_op("mul"), 2, 1), "func-div": (_extern_op("div"), 2, 1),
          "func-term": (lambda mem, a: (TERMINATED, [1234]), 0, 1),
          "func-fail": (lambda mem, a: (HOST_FAILED, [5678]), 0, 1)}


def register_extern(ctx):
    for name, (fn, np_, nr) in EXTERN.items():
        ctx.add_host_function("extern", name, fn, np_, nr)


# ---- the reference externref test's import module "extern_module"
# (test/externref/ExternrefTest.cpp:20-70, registered at :172-211): the externref names a
# host object the function calls. Handles as in the oracle: 1 = AddClass, 2 = MulFunc,
# 3 = SquareStruct; a null or other handle fails the call (HostFuncFailed).
EXT_ADD, EXT_MUL, EXT_SQUARE = 1, 2, 3


def _ext_obj(kind, f, nargs):
    def g(mem, a):
        if a[0] & 0xFFFFFFFF != kind:
            return HOST_FAILED, []
        return 0, [f(*[x & 0xFFFFFFFF for x in a[1:1 + nargs]]) & 0xFFFFFFFF]
    return g


EXTERN_MODULE = {"class_add": (_ext_obj(EXT_ADD, lambda x, y: x + y, 2), 3, 1),
                 "func_mul": (_ext_obj(EXT_MUL, lambda x, y: x * y, 2), 3, 1),
                 "functor_square": (_ext_obj(EXT_SQUARE, lambda x: x * x, 1), 2, 1)}


def register_extern_module(ctx):
    for name, (fn, np_, nr) in EXTERN_MODULE.items():
        ctx.add_host_function("extern_module", name, fn, np_, nr)


def register(ctx):
    for name, (fn, np_, nr) in ENV.items():
        ctx.add_host_function("env", name, fn, np_, nr)


# ---- the same functions on the host emulator's inline host hook (wb_emu_set_host)
SIGS = {"add_i64": ("ll", "l"), "mem_sum": ("ii", "i"), "mem_fill": ("iii", ""),
        "fail": ("i", "i"), "exit": ("i", ""), "mix": ("id", "d")}
_CELLS = {"i": 1, "f": 1, "l": 2, "d": 2}


class _EmuMem:
    def __init__(self, ptr, size):
        self.ptr, self.size = ptr, size

    def read(self, off, n):
        import ctypes
        if off + n > self.size:
            raise WasmEdgeError(MEM_OOB, "read")
        return ctypes.string_at(self.ptr + off, n)

    def write(self, off, data):
        import ctypes
        if off + len(data) > self.size:
            raise WasmEdgeError(MEM_OOB, "write")
        ctypes.memmove(self.ptr + off, bytes(data), len(data))


def emu_host(import_names):
    """A wb_emu_host_t callback serving the module's imports (listed in import order)."""
    import ctypes
    proto = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                             ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                             ctypes.c_void_p, ctypes.c_uint64)

    def cb(inst, func, args, rets, mem, size):
        name = import_names[func]
        fn = ENV[name][0]
        ps, rs = SIGS[name]
        vals, at = [], 0
        for t in ps:
            v = 0
            for q in range(_CELLS[t]):
                v |= args[at] << (32 * q)
                at += 1
            vals.append(v)
        code, res = fn(_EmuMem(mem, size), vals)
        if code:
            return code
        at = 0
        for t, v in zip(rs, res):
            for q in range(_CELLS[t]):
                rets[at] = (v >> (32 * q)) & 0xFFFFFFFF
                at += 1
        return 0
    return proto(cb)
