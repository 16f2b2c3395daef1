"""The reference's externref test module (test/externref/externrefTestData/funcs.wasm,
fixture tests/golden/externref_funcs.wasm) and its expected answers
(test/externref/ExternrefTest.cpp:308-356):

* call_add(&AddClass, 1234, 5678)                 = 6912
* call_mul(&MulFunc, 789, 4321)                   = 3409269
* call_square(&SquareStruct, 8256)                = 68161536
* call_add_square(&AddClass, &SquareStruct, 210, 654) = 746496

Externref parameters of exported functions pass straight into imports of the host module
"extern_module" (tests/hostfuncs.py, oracle host_call), so every call goes through the
host-import yield path. Handles: 1 = AddClass, 2 = MulFunc, 3 = SquareStruct; a null or
mismatched handle fails the call with HostFuncFailed (0x8D) -- undefined behaviour in the
C++ test, a defined per-lane trap here and in the oracle."""
import pytest

import hostfuncs
import oracle_py as O
from conftest import golden
from helpers import compare

I32, EXTERNREF = 0x7F, 0x6F
NULL = 0xFFFFFFFF
ADD, MUL, SQ = hostfuncs.EXT_ADD, hostfuncs.EXT_MUL, hostfuncs.EXT_SQUARE
KATS = [("call_add", [ADD, 1234, 5678], [EXTERNREF, I32, I32], 6912),
        ("call_mul", [MUL, 789, 4321], [EXTERNREF, I32, I32], 3409269),
        ("call_square", [SQ, 8256], [EXTERNREF, I32], 68161536),
        ("call_add_square", [ADD, SQ, 210, 654], [EXTERNREF, EXTERNREF, I32, I32], 746496)]
N = 200


def _wasm():
    return golden("externref_funcs.wasm")


def test_externref_oracle_kats():
    m = O.Module(_wasm())
    inst = O.Instance(m)
    assert inst.error == 0
    for fn, args, _, want in KATS:
        code, vals, cnt, _ = inst.invoke(fn, args)
        assert (code, vals) == (0, [want]), fn
    # a null / mismatched object fails the host call
    assert inst.invoke("call_add", [NULL, 1, 2])[0] == hostfuncs.HOST_FAILED
    assert inst.invoke("call_square", [MUL, 3])[0] == hostfuncs.HOST_FAILED


def _rows(fn, n):
    """Per-lane handles (mostly right, some null / wrong) and operands."""
    rows = []
    for i in range(n):
        x, y = (i * 2654435761) & 0xFFFFFFFF, (i * 40503 + 7) & 0xFFFFFFFF
        bad = i % 9 == 4
        if fn == "call_add":
            rows.append([NULL if bad else ADD, x, y])
        elif fn == "call_mul":
            rows.append([SQ if bad else MUL, x, y])
        elif fn == "call_square":
            rows.append([NULL if bad else SQ, x])
        else:
            rows.append([ADD, MUL if bad else SQ, x, y] if i % 2 else [NULL if bad else ADD, SQ, x, y])
    return rows


@pytest.mark.gpu
def test_gpu_externref_reference_answers(built):
    from wasmedge_amd import batch
    ctx = batch.BatchContext(_wasm(), N, device=0)
    try:
        hostfuncs.register_extern_module(ctx)
        for fn, args, types, want in KATS:
            rets, st, cnt = ctx.execute(fn, batch.make_values([args] * N, types), 1)
            assert (st == 0).all(), fn
            assert [int(r[0]) for r in batch.ret_ints(rets)] == [want] * N, fn
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_externref_per_lane_vs_oracle(built):
    """Per-lane externrefs (including null and mismatched objects) vs the oracle:
    status, result and instruction count of every lane."""
    from wasmedge_amd import batch
    m = O.Module(_wasm())
    ctx = batch.BatchContext(_wasm(), N, device=0)
    try:
        hostfuncs.register_extern_module(ctx)
        for fn, _, types, _ in KATS:
            rows = _rows(fn, N)
            ref = [O.Instance(m).invoke(fn, r) for r in rows]
            assert any(r[0] for r in ref) and any(not r[0] for r in ref)
            rets, st, cnt = ctx.execute(fn, batch.make_values(rows, types), 1)
            ints = batch.ret_ints(rets)
            got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(N)]
            assert compare(ref, got, st, cnt, None, [I32], check_hash=False) == [], fn
    finally:
        ctx.close()


# ---- test/externref/externrefTestData/stl.wasm (ExternrefTest.cpp:360-465): externrefs
# to host C++ containers; the host functions mutate them. Here every lane gets its own
# containers in a host object registry (handle = index), and each lane must see exactly
# the reference's expected contents after each call: one host call per lane, in order.

class _Objects:
    def __init__(self):
        self.objs = []

    def new(self, o):
        self.objs.append(o)
        return len(self.objs) - 1

    def __getitem__(self, h):
        return self.objs[h & 0xFFFFFFFF]


def _stl_module(reg, calls):
    def rec(name, f, nres):
        def g(mem, a):
            calls.append((name, mem.instance))
            r = f(*a)
            return 0, ([r & 0xFFFFFFFF] if nres else [])
        return g

    def vsum(b, e):
        (vb, ib), (ve, ie) = reg[b], reg[e]
        assert vb == ve
        return sum(reg[vb][ib:ie])

    return {
        "stl_ostream_str": (rec("ostream_str", lambda s, x: reg[s].append(reg[x]), 0), 2, 0),
        "stl_ostream_u32": (rec("ostream_u32", lambda s, v: reg[s].append(str(v & 0xFFFFFFFF)), 0), 2, 0),
        "stl_map_insert": (rec("map_insert", lambda m, k, v: reg[m].__setitem__(reg[k], reg[v]), 0), 3, 0),
        "stl_map_erase": (rec("map_erase", lambda m, k: reg[m].pop(reg[k], None), 0), 2, 0),
        "stl_set_insert": (rec("set_insert", lambda s, v: reg[s].add(v & 0xFFFFFFFF), 0), 2, 0),
        "stl_set_erase": (rec("set_erase", lambda s, v: reg[s].discard(v & 0xFFFFFFFF), 0), 2, 0),
        "stl_vector_push": (rec("vector_push", lambda v, x: reg[v].append(x & 0xFFFFFFFF), 0), 2, 0),
        "stl_vector_sum": (rec("vector_sum", vsum, 1), 2, 1),
    }


def test_externref_stl_oracle_counts():
    m = O.Module(golden("externref_stl.wasm"))
    inst = O.Instance(m)
    assert inst.error == 0
    for fn, args in [("call_ostream_str", [0, 1]), ("call_map_insert", [0, 1, 2]),
                     ("call_vector_sum", [0, 1])]:
        code, _, cnt, _ = inst.invoke(fn, args)
        assert code == 0 and cnt == len(args) + 2, fn     # local.get x k, call, end


@pytest.mark.gpu
def test_gpu_externref_stl_reference_answers(built):
    from wasmedge_amd import batch
    n = 96
    wasm = golden("externref_stl.wasm")
    m = O.Module(wasm)
    reg, calls = _Objects(), []
    lanes = []
    for i in range(n):
        L = {"ss": reg.new([]), "str": reg.new("hello world!"), "key": reg.new("one"),
             "val": reg.new("1"), "map": reg.new({}), "set": reg.new(set()),
             "vec": reg.new([10, 20, 30, 40, 50, 60, 70, 80, 90])}
        lanes.append(L)
    ctx = batch.BatchContext(wasm, n, device=0)
    E = EXTERNREF

    def run(fn, rows, types, nres=0):
        calls.clear()
        ref = [O.Instance(m).invoke(fn, r) for r in rows]
        rets, st, cnt = ctx.execute(fn, batch.make_values(rows, types), nres)
        assert (st == 0).all(), fn
        assert [int(c) for c in cnt] == [r[2] for r in ref], fn
        assert sorted(c[1] for c in calls) == list(range(n)), fn   # once per lane
        return rets

    try:
        for name, (fn, np_, nr) in _stl_module(reg, calls).items():
            ctx.add_host_function("extern_module", name, fn, np_, nr)
        run("call_ostream_str", [[L["ss"], L["str"]] for L in lanes], [E, E])
        assert all("".join(reg[L["ss"]]) == "hello world!" for L in lanes)
        run("call_ostream_u32", [[L["ss"], 123456] for L in lanes], [E, I32])
        assert all("".join(reg[L["ss"]]) == "hello world!123456" for L in lanes)
        run("call_map_insert", [[L["map"], L["key"], L["val"]] for L in lanes], [E, E, E])
        assert all(reg[L["map"]] == {"one": "1"} for L in lanes)
        run("call_map_erase", [[L["map"], L["key"]] for L in lanes], [E, E])
        assert all(reg[L["map"]] == {} for L in lanes)
        run("call_set_insert", [[L["set"], 123456] for L in lanes], [E, I32])
        for L in lanes:
            reg[L["set"]].add(3456)
        run("call_set_erase", [[L["set"], 3456] for L in lanes], [E, I32])
        assert all(reg[L["set"]] == {123456} for L in lanes)
        run("call_vector_push", [[L["vec"], 100] for L in lanes], [E, I32])
        assert all(len(reg[L["vec"]]) == 10 and reg[L["vec"]][9] == 100 for L in lanes)
        rows = [[reg.new((L["vec"], 3)), reg.new((L["vec"], 8))] for L in lanes]
        rets = run("call_vector_sum", rows, [E, E], 1)
        assert [int(r[0]) for r in batch.ret_ints(rets)] == [40 + 50 + 60 + 70 + 80] * n
    finally:
        ctx.close()


# ---- 64-bit externref values: the reference's externrefs are host pointers
# (WasmEdge_ValueGenExternRef(void*), wasmedge.h:254,318; ExternrefTest.cpp passes &AddClass).
# Values from 2^31 up cross the boundary unchanged -- arguments, results, host-function
# arguments and results, table and global reads and writes -- while the device carries a
# 32-bit handle the context interns (batch_ctx.h xref_in / xref_out).
def _keep_wasm():
    from wasmedge_amd.wat import assemble
    return assemble(r"""
(module
  (import "env" "echo" (func $echo (param externref) (result externref)))
  (table $t 4 externref)
  (global $g (mut externref) (ref.null extern))
  (export "t" (table $t))
  (export "g" (global $g))
  (func (export "keep") (param $a externref) (param $b externref) (result externref)
    (table.set $t (i32.const 1) (local.get $a))
    (global.set $g (local.get $b))
    (call $echo (table.get $t (i32.const 1))))
  (func (export "peek") (result externref) (table.get $t (i32.const 2)))
)
""")


def _ptr(i, k):
    """A pointer-like 64-bit value, distinct per (lane, k)."""
    return 0x00007F3A5C000000 + (i * 4 + k) * 48


@pytest.mark.gpu
def test_gpu_externref_64bit_values(built):
    from wasmedge_amd import batch
    n = 130
    seen = {}

    def echo(mem, a):
        seen[mem.instance] = a[0]
        return 0, [a[0]]

    ctx = batch.BatchContext(_keep_wasm(), n, device=0)
    try:
        ctx.add_host_function("env", "echo", echo, 1, 1)
        rows = [[_ptr(i, 0), NULL if i % 5 == 3 else _ptr(i, 1)] for i in range(n)]
        rets, st, cnt = ctx.execute("keep", batch.make_values(rows, [EXTERNREF, EXTERNREF]), 1)
        assert (st == 0).all()
        assert [int(r[0]) for r in batch.ret_ints(rets)] == [r[0] for r in rows]
        assert seen == {i: rows[i][0] for i in range(n)}        # the host saw the pointer
        for i in (0, 3, 64, 129):
            assert ctx.table_get("t", i, 1) == (rows[i][0], EXTERNREF)
            assert ctx.global_get("g", i) == (rows[i][1], EXTERNREF)
            assert ctx.table_get("t", i, 0) == (NULL, EXTERNREF)
        # written by the host through the API, read back by the module and the API
        for i in range(n):
            ctx.table_set("t", i, 2, _ptr(i, 2), EXTERNREF)
        ctx.global_set("g", 7, _ptr(7, 3), EXTERNREF)
        rets, st, cnt = ctx.execute("peek", batch.make_values([[]] * n, []), 1)
        assert (st == 0).all()
        assert [int(r[0]) for r in batch.ret_ints(rets)] == [_ptr(i, 2) for i in range(n)]
        assert ctx.global_get("g", 7) == (_ptr(7, 3), EXTERNREF)
        # small values stay their own device refs (the handles the tests above use)
        rets, st, cnt = ctx.execute("keep", batch.make_values([[5, 6]] * n, [EXTERNREF, EXTERNREF]), 1)
        assert [int(r[0]) for r in batch.ret_ints(rets)] == [5] * n
        assert ctx.global_get("g", 0) == (6, EXTERNREF)
    finally:
        ctx.close()
