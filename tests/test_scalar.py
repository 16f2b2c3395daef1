"""Scalar numerics and trap matrix (VERDICT r1 "next #2").

Every one-byte numeric opcode and the 0xFC trunc_sat family on special operands
(tests/scalar_cases.py), every trap-capable scalar op (div/rem: 0x84 DivideByZero, 0x85
IntegerOverflow; trunc: 0x86 InvalidConvToInt, 0x85 out of range), and the control traps
0x87 (table.get), 0x88, 0x89, 0x8A, 0x8B, 0x8C plus the device's 0xB0 (call stack
exhausted). Compared EXACTLY against the oracle: NaN results bit for bit (return values
and the memory hash, which covers every op's stored result), and the memory of trapped
instances too.

NaN payload rules are those of the reference as g++ -O2 compiles it on x86-64
(tools/nan_probe.cpp): add/mul keep the first (lhs) NaN operand quieted, ceil/floor/trunc
return a NaN unchanged, the rest quiet it / produce the negative default NaN. They are
pinned to the compiler's code for the reference's expression shapes, not to a reference
binary (none can be built here): beyond that, parity unpinned.

On the GPU each case runs through the three execution engines: the threaded core with
frames in VGPRs (default at these sizes), the threaded core with LDS frames
(WB_VFRAME=0), the compiled per-op step (WB_THREADED=0), and the compiled step over
frames in HBM (WB_HBMFRAME=1, the mode of frames too large for LDS)."""
import pytest

import oracle_py as O
import scalar_cases as S
from helpers import compare, emu_run, gpu_run

I32, I64 = 0x7F, 0x7E
ROWS = [[i] for i in range(S.N * S.N)]
TRAP_ROWS = [[op, i] for op in range(len(S.trap_ops())) for i in range(S.N * S.N)]
CTRL_ROWS = [[c, x] for c in range(8) for x in list(range(12)) + [40, 100, 300, 1000]]
ENGINES = {"vframe": {"WB_VFRAME": "1"}, "ldsframe": {"WB_VFRAME": "0"},
           "step": {"WB_THREADED": "0"}, "hbmframe": {"WB_HBMFRAME": "1"}}
TRAP_CODES = {0x84, 0x85, 0x86}


def _ref(wasm, func, rows):
    m = O.Module(wasm)
    return [m.run(func, r) for r in rows]


def test_module_names_every_scalar_opcode():
    assert S.ops_covered() == set(S.scalar_ops())
    assert len(S.scalar_ops()) == 128 + 8


def test_oracle_trap_matrix_covers_codes():
    ref = _ref(S.scalar_wasm(), "trap", TRAP_ROWS)
    assert {r[0] for r in ref} == {0} | TRAP_CODES
    ctrl = _ref(S.ctrl_wasm(), "ctrl", CTRL_ROWS)
    assert {r[0] for r in ctrl} == {0, 0x87, 0x88, 0x89, 0x8A, 0x8B, 0x8C}


@pytest.mark.parametrize("func,rows,pt", [("scalar", ROWS, [I32]), ("trap", TRAP_ROWS, [I32, I32])],
                         ids=["scalar", "trap"])
def test_emulator_scalar_exact(built, func, rows, pt):
    wasm = S.scalar_wasm()
    ref = _ref(wasm, func, rows)
    got = emu_run(wasm, func, rows, pt, [I64])
    assert compare(ref, *got, [I64], exact=True) == []


def _ctrl_check(ref, got, depth_limited):
    """Recursion (case 4) may exhaust the device call stack (0xB0) where the reference's
    stack grows without bound (stackmgr.h:44-47); every other instance is exact."""
    rets, st, cnt, h = got
    exhausted = 0
    keep = []
    for i, r in enumerate(ref):
        if CTRL_ROWS[i][0] == 4 and int(st[i]) == 0xB0:
            assert depth_limited and CTRL_ROWS[i][1] >= 40, CTRL_ROWS[i]
            exhausted += 1
            keep.append((0xB0, [], int(cnt[i]), int(h[i])))
        else:
            keep.append(r)
    assert compare(keep, rets, st, cnt, h, [I32], exact=True) == []
    return exhausted


def test_emulator_ctrl_traps(built):
    wasm = S.ctrl_wasm()
    ref = _ref(wasm, "ctrl", CTRL_ROWS)
    got = emu_run(wasm, "ctrl", CTRL_ROWS, [I32, I32], [I32], gs_depth=64)
    assert _ctrl_check(ref, got, True) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("engine", sorted(ENGINES))
def test_gpu_scalar_exact(built, monkeypatch, engine):
    for k, v in ENGINES[engine].items():
        monkeypatch.setenv(k, v)
    wasm = S.scalar_wasm()
    for func, rows, pt in (("scalar", ROWS, [I32]), ("trap", TRAP_ROWS, [I32, I32])):
        ref = _ref(wasm, func, rows)
        got = gpu_run(wasm, func, rows, pt, [I64], device=0)
        assert compare(ref, *got, [I64], exact=True) == [], func


@pytest.mark.gpu
@pytest.mark.parametrize("engine", sorted(ENGINES))
def test_gpu_ctrl_traps(built, monkeypatch, engine):
    for k, v in ENGINES[engine].items():
        monkeypatch.setenv(k, v)
    wasm = S.ctrl_wasm()
    ref = _ref(wasm, "ctrl", CTRL_ROWS)
    got = gpu_run(wasm, "ctrl", CTRL_ROWS, [I32, I32], [I32], device=0, call_stack_cells=64)
    assert _ctrl_check(ref, got, True) > 0
