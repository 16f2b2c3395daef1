"""The reference's C-API test module (test/api/apiTestData/test.wasm, fixture
tests/golden/apitest.wasm) and its expected answers (test/api/APIUnitTest.cpp):

* func-mul-2(123, 456) = (246, 912)                                  (:1170-1180)
* func-host-{add,sub,mul,div} through externrefs set in table tab-ext with
  WasmEdge_TableInstanceSetData: 777+223 = 1000, 123-456 = -333, -30*-66 = 1980,
  -9999/1234 = -8                                                     (:1225-1275)
* exported globals glob-mut-i32 = 142, glob-const-f32 = 789.12         (test.wat:70-71)
* func-call-indirect over table tab-func (elem at 2: func-1..func-4)  (test.wat:37-40,61-62)

Two tables (funcref + externref), an exported table and externref-typed host imports
exercise the per-lane table mode, the table/global C-ABI and the host-import yield path;
the oracle (with the same "extern" host module) checks counts and per-lane variants."""
import struct

import numpy as np
import pytest

import hostfuncs
import oracle_py as O
from conftest import golden
from helpers import compare, emu_run

I32, F32, FUNCREF, EXTERNREF = 0x7F, 0x7D, 0x70, 0x6F
N = 130


def _wasm():
    return golden("apitest.wasm")


def test_apitest_oracle_kats():
    m = O.Module(_wasm())
    inst = O.Instance(m)
    assert inst.error == 0
    code, vals, _, _ = inst.invoke("func-mul-2", [123, 456])
    assert (code, vals) == (0, [246, 912])
    assert inst.global_get(0) == 142
    assert inst.global_get(1) == struct.unpack("<I", struct.pack("<f", 789.12))[0]
    for k in range(4):
        assert inst.table_set(1, k, 7) == 0
    assert inst.table_set(1, 10, 7) == 0x87
    for fn, tv, p, want in [("func-host-add", 777, 223, 1000), ("func-host-sub", 123, 456, -333),
                            ("func-host-mul", -30, -66, 1980), ("func-host-div", -9999, 1234, -8)]:
        O.set_extern_value(7, tv)
        code, vals, _, _ = inst.invoke(fn, [p & 0xFFFFFFFF])
        assert code == 0 and vals == [want & 0xFFFFFFFF], fn
    # call_indirect: 0,1 and 6..9 null (UninitializedElement), 10+ UndefinedElement
    got = [inst.invoke("func-call-indirect", [i])[:2] for i in range(12)]
    assert got == [(0x8A, [])] * 2 + [(0, [k]) for k in (1, 2, 3, 4)] + [(0x8A, [])] * 4 + \
        [(0x8B, [])] * 2


def test_apitest_emulator():
    """Exports that call no import, through the kernel's step code on the host."""
    m = O.Module(_wasm())
    rows = [[i % 13] for i in range(40)]
    ref = [O.Instance(m).invoke("func-call-indirect", r) for r in rows]
    rets, st, cnt, h = emu_run(_wasm(), "func-call-indirect", rows, [I32], [I32])
    assert compare(ref, rets, st, cnt, h, [I32]) == []
    rows = [[i * 7919, 3 - i] for i in range(40)]
    ref = [O.Instance(m).invoke("func-mul-2", r) for r in rows]
    rets, st, cnt, h = emu_run(_wasm(), "func-mul-2", rows, [I32, I32], [I32, I32])
    assert compare(ref, rets, st, cnt, h, [I32, I32]) == []


def _ints(rets, st):
    from wasmedge_amd import batch
    ints = batch.ret_ints(rets)
    return [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(st))]


@pytest.mark.gpu
def test_gpu_apitest_reference_answers(built):
    from wasmedge_amd import batch
    ctx = batch.BatchContext(_wasm(), N, device=0)
    try:
        hostfuncs.register_extern(ctx)
        rets, st, cnt = ctx.execute("func-mul-2", batch.make_values([[123, 456]] * N, [I32, I32]), 2)
        assert (st == 0).all() and _ints(rets, st) == [[246, 912]] * N
        assert ctx.global_get("glob-mut-i32", 5) == (142, I32)
        assert ctx.global_get("glob-const-f32", 129) == (struct.unpack("<I", struct.pack("<f", 789.12))[0], F32)
        assert ctx.table_size("tab-ext", 0) == 10 and ctx.table_size("tab-func", 77) == 10
        assert ctx.table_get("tab-func", 3, 2) == (6, FUNCREF)       # func-1 = function 6
        assert ctx.table_get("tab-ext", 3, 0) == (batch.REF_NULL, EXTERNREF)
        for k in range(4):
            ctx.table_set("tab-ext", None, k, 7, EXTERNREF)
        with pytest.raises(batch.WasmEdgeError) as e:
            ctx.table_set("tab-ext", None, 10, 7, EXTERNREF)
        assert e.value.code == 0x87
        with pytest.raises(batch.WasmEdgeError) as e:
            ctx.table_set("tab-ext", 0, 1, 7, FUNCREF)
        assert e.value.code == 0x8E
        for fn, tv, p, want in [("func-host-add", 777, 223, 1000), ("func-host-sub", 123, 456, -333),
                                ("func-host-mul", -30, -66, 1980), ("func-host-div", -9999, 1234, -8)]:
            hostfuncs.EXTERN_VALUES[7] = tv
            rets, st, cnt = ctx.execute(fn, batch.make_values([[p & 0xFFFFFFFF]] * N, [I32]), 1)
            assert (st == 0).all() and _ints(rets, st) == [[want & 0xFFFFFFFF]] * N, fn
        rets, st, cnt = ctx.execute("func-call-indirect",
                                    batch.make_values([[i % 12] for i in range(N)], [I32]), 1)
        want = {0: 0x8A, 1: 0x8A, 6: 0x8A, 7: 0x8A, 8: 0x8A, 9: 0x8A, 10: 0x8B, 11: 0x8B}
        for i in range(N):
            k = i % 12
            assert int(st[i]) == want.get(k, 0)
            if k in (2, 3, 4, 5):
                assert int(batch.ret_ints(rets)[i][0]) == k - 1
        ctx.global_set("glob-mut-i32", None, 9, I32)
        ctx.global_set("glob-const-f32", None, 0, F32)     # constant: ignored
        assert ctx.global_get("glob-mut-i32", 64) == (9, I32)
        assert ctx.global_get("glob-const-f32", 64)[0] == struct.unpack("<I", struct.pack("<f", 789.12))[0]
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_apitest_per_lane_externrefs(built):
    """Per-instance externrefs and tables vs the oracle (counts and results)."""
    from wasmedge_amd import batch
    vals = {3: 777, 4: -30, 5: -9999, 6: 41}
    m = O.Module(_wasm())
    insts = [O.Instance(m) for _ in range(N)]
    ctx = batch.BatchContext(_wasm(), N, device=0)
    try:
        hostfuncs.register_extern(ctx)
        hostfuncs.EXTERN_VALUES.clear()
        hostfuncs.EXTERN_VALUES.update(vals)
        for h, v in vals.items():
            O.set_extern_value(h, v)
        for i in range(N):
            if i % 5 == 4:
                continue                         # left null: the host function fails
            ctx.table_set("tab-ext", i, i % 4, 3 + i % 4, EXTERNREF)
            assert insts[i].table_set(1, i % 4, 3 + i % 4) == 0
        for fn in ("func-host-add", "func-host-sub", "func-host-mul", "func-host-div"):
            rows = [[(i * 37 - 500) & 0xFFFFFFFF] for i in range(N)]
            ref = [inst.invoke(fn, r) for inst, r in zip(insts, rows)]
            rets, st, cnt = ctx.execute(fn, batch.make_values(rows, [I32]), 1)
            assert compare(ref, _ints(rets, st), st, cnt, ctx.memory_hash(), [I32]) == [], fn
    finally:
        ctx.close()
