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
