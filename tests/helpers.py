"""Shared test helpers: run a module on the oracle and on the device/emulator and
compare return bits, trap codes, instruction counts and memory hashes."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU_PATH = os.environ.get("WB_EMU_LIB") or os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch_emu.so")
_emu = None

CELLS = {0x7F: 1, 0x7E: 2, 0x7D: 1, 0x7C: 2, 0x7B: 4, 0x70: 1, 0x6F: 1}


def emu_lib():
    global _emu
    if _emu is None:
        E = ctypes.CDLL(EMU_PATH)
        E.wb_emu_last_error.restype = ctypes.c_char_p
        E.wb_emu_execute.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                     ctypes.c_uint32] + [ctypes.c_void_p] * 5 + \
            [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        E.wb_emu_set_host.argtypes = [ctypes.c_void_p]
        E.wb_emu_set_cost_limit.argtypes = [ctypes.c_uint64]
        E.wb_emu_set_cost_table.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        E.wb_emu_add_import.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_uint32] * 6 + \
            [ctypes.c_void_p]
        E.wb_emu_get_costs.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        cpp = ctypes.POINTER(ctypes.c_char_p)
        E.wb_emu_set_wasi.argtypes = [ctypes.c_int, cpp, ctypes.c_uint32, cpp, ctypes.c_uint32]
        E.wb_emu_set_wasi_preopens.argtypes = [cpp, ctypes.c_uint32]
        E.wb_emu_set_instance_args.argtypes = [ctypes.c_uint32, cpp, ctypes.c_uint32]
        E.wb_emu_set_wasi_deterministic.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        E.wb_emu_wasi_output.restype = ctypes.c_uint32
        E.wb_emu_wasi_output.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32]
        E.wb_emu_wasi_exit_code.restype = ctypes.c_uint32
        E.wb_emu_wasi_exit_code.argtypes = [ctypes.c_uint32]
        E.wb_emu_disasm.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                    ctypes.c_uint32]
        _emu = E
    return _emu


def to_cells(args, types):
    out = []
    for a, t in zip(args, types):
        v = int(a) & ((1 << 128) - 1)
        for q in range(CELLS[t]):
            out.append((v >> (32 * q)) & 0xFFFFFFFF)
    return out


def from_cells(cells, types):
    vals, at = [], 0
    for t in types:
        v = 0
        for q in range(CELLS[t]):
            v |= int(cells[at]) << (32 * q)
            at += 1
        vals.append(v)
    return vals


def emu_run(wasm, func, arg_rows, ptypes, rtypes, max_pages=0, gs_depth=0, max_steps=0,
            host=None, cost_limit=0, cost_table=None, costs_out=None, tail_call=False,
            multi_memory=False):
    """host: a wb_emu_host_t ctypes callback serving imports inline (hostfuncs.emu_host);
    cost_limit: gas limit (0 = none) with cost_table (list by OpCode, None = unit costs);
    costs_out: a list that receives each instance's gas total; tail_call / multi_memory: the
    TailCall / MultiMemories proposals."""
    E = emu_lib()
    E.wb_emu_set_tail_call(1 if tail_call else 0)
    E.wb_emu_set_multi_memory(1 if multi_memory else 0)
    E.wb_emu_set_host(host)
    E.wb_emu_set_cost_limit(cost_limit)
    if cost_table is None:
        E.wb_emu_set_cost_table(None, 0)
    else:
        tab = np.ascontiguousarray(cost_table, np.uint64)
        E.wb_emu_set_cost_table(tab.ctypes.data, len(tab))
    n = len(arg_rows)
    pc = sum(CELLS[t] for t in ptypes)
    rc = sum(CELLS[t] for t in rtypes)
    params = np.zeros((n, max(pc, 1)), np.uint32)
    for i, row in enumerate(arg_rows):
        params[i, :pc] = to_cells(row, ptypes)
    res = np.zeros((n, max(rc, 1)), np.uint32)
    st = np.zeros(n, np.uint8)
    cnt = np.zeros(n, np.uint64)
    h = np.zeros(n, np.uint64)
    e = E.wb_emu_execute(wasm, len(wasm), func.encode(), n, params.ctypes.data,
                         res.ctypes.data, st.ctypes.data, cnt.ctypes.data, h.ctypes.data,
                         max_pages, gs_depth, max_steps)
    if e:
        raise RuntimeError("emu error 0x%x: %s" % (e, E.wb_emu_last_error().decode()))
    if costs_out is not None:
        c = np.zeros(n, np.uint64)
        E.wb_emu_get_costs(c.ctypes.data, n)
        costs_out[:] = [int(x) for x in c]
    rets = [from_cells(res[i], rtypes) if st[i] == 0 else [] for i in range(n)]
    return rets, st, cnt, h


def emu_set_imports(imports):
    """Provided tables / memories / globals for the emulator (dicts as oracle_py.set_imports)."""
    E = emu_lib()
    E.wb_emu_clear_imports()
    for i in imports or []:
        v = int(i.get("value", 0)) & ((1 << 128) - 1)
        cells = (ctypes.c_uint32 * 4)(*[(v >> (32 * q)) & 0xFFFFFFFF for q in range(4)])
        mx = i.get("max")
        E.wb_emu_add_import(i["module"].encode(), i["name"].encode(), i["kind"], i.get("type", 0),
                            1 if i.get("mut") else 0, i.get("min", 0), mx or 0,
                            0 if mx is None else 1, ctypes.cast(cells, ctypes.c_void_p))


def emu_set_wasi(on, args=(), envs=(), preopens=(), instance_args=None, deterministic=None):
    """The emulator's copy of the library's WASI subset (wasi_impl.h); instance_args:
    {instance: its own args} for the next run; deterministic: (seed, clock_ns)."""
    def arr(v):
        return (ctypes.c_char_p * max(len(v), 1))(*[x.encode() for x in v])
    E = emu_lib()
    E.wb_emu_set_wasi(1 if on else 0, arr(list(args)), len(args), arr(list(envs)), len(envs))
    E.wb_emu_set_wasi_preopens(arr(list(preopens)), len(preopens))
    E.wb_emu_clear_instance_args()
    seed, clock = deterministic or (0, 0)
    E.wb_emu_set_wasi_deterministic(1 if deterministic else 0, seed, clock)
    for i, a in (instance_args or {}).items():
        E.wb_emu_set_instance_args(i, arr(list(a)), len(a))


def emu_wasi_output(inst, fd):
    E = emu_lib()
    n = E.wb_emu_wasi_output(inst, fd, None, 0)
    buf = ctypes.create_string_buffer(max(n, 1))
    E.wb_emu_wasi_output(inst, fd, buf, n)
    return buf.raw[:n]


def disasm(wasm):
    E = emu_lib()
    buf = ctypes.create_string_buffer(1 << 22)
    E.wb_emu_disasm(wasm, len(wasm), buf, len(buf))
    return buf.value.decode()


def canon(v, t):
    """Canonicalise NaN payloads as the spec permits (f32/f64 results only)."""
    if t == 0x7D and (v & 0x7FFFFFFF) > 0x7F800000:
        return "nan32"
    if t == 0x7C and (v & 0x7FFFFFFFFFFFFFFF) > 0x7FF0000000000000:
        return "nan64"
    return v


def oracle_run(mod, func, arg_rows):
    out = []
    for row in arg_rows:
        code, vals, cnt, h = mod.run(func, row)
        out.append((code, vals, cnt, h))
    return out


def gpu_run(wasm, func, arg_rows, ptypes, rtypes, **kw):
    from wasmedge_amd import batch
    ctx = batch.BatchContext(wasm, len(arg_rows), **kw)
    try:
        vals = batch.make_values(arg_rows, ptypes)
        rets, st, cnt = ctx.execute(func, vals, len(rtypes))
        h = ctx.memory_hash()
        ints = batch.ret_ints(rets)
        rows = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(arg_rows))]
        return rows, st, cnt, h
    finally:
        ctx.close()


def compare(oracle_rows, rets, st, cnt, h, rtypes, check_hash=True, exact=False):
    """Differences between oracle rows (code, values, count, memhash) and a device /
    emulator run. exact=True compares NaN return payloads bit for bit (no canon) and the
    memory hash of trapped instances too (memory as the trap left it)."""
    bad = []
    for i, (code, vals, ocnt, oh) in enumerate(oracle_rows):
        if int(st[i]) != code:
            bad.append((i, "status", code, int(st[i])))
            continue
        if int(cnt[i]) != ocnt:
            bad.append((i, "count", ocnt, int(cnt[i])))
        if code == 0:
            a = list(vals) if exact else [canon(v, t) for v, t in zip(vals, rtypes)]
            b = list(rets[i]) if exact else [canon(v, t) for v, t in zip(rets[i], rtypes)]
            if a != b:
                bad.append((i, "ret", vals, rets[i]))
        if check_hash and (code == 0 or exact) and int(h[i]) != oh:
            bad.append((i, "memhash", oh, int(h[i])))
    return bad
