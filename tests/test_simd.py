"""SIMD128 parity: every 0xFD opcode of the reference, on random and
special-value operands, device / host emulator vs the oracle -- return bits, trap codes,
instruction counts and final-memory hashes. FP results are compared bit for bit (the
memory hash covers NaN payloads exactly; no canonicalisation is applied there)."""
import pytest

import oracle_py as O
from helpers import compare, emu_run, gpu_run, oracle_run
from simd_cases import I32, I64, all_simd_ops, ops_covered, simd_wasm

ROWS = [[i] for i in range(96)] + [[1000003], [0x7FFFFFFF], [0xFFFFFFFF]]
# lane_oob(addr, which): the lane forms at the page end and with an EA overflow
OOB_ROWS = [[a, w] for a in (0, 65520, 65528, 65532, 65534, 65535, 0xFFFFFFF0, 0xFFFFFFFE)
            for w in range(4)]


def test_module_names_every_simd_opcode():
    missing = all_simd_ops() - ops_covered()
    assert not missing, sorted(missing)


def test_simd_emulator_parity(built):
    wasm = simd_wasm()
    m = O.Module(wasm)
    ref = oracle_run(m, "simd", ROWS)
    assert all(r[0] == 0 for r in ref)
    rets, st, cnt, h = emu_run(wasm, "simd", ROWS, [I32], [I64])
    assert compare(ref, rets, st, cnt, h, [I64], exact=True) == []
    ref = oracle_run(m, "lane_oob", OOB_ROWS)
    assert {r[0] for r in ref} == {0, 0x88}
    rets, st, cnt, h = emu_run(wasm, "lane_oob", OOB_ROWS, [I32, I32], [I32])
    assert compare(ref, rets, st, cnt, h, [I32], exact=True) == []


@pytest.mark.gpu
def test_gpu_simd_parity(built):
    wasm = simd_wasm()
    m = O.Module(wasm)
    ref = oracle_run(m, "simd", ROWS)
    rets, st, cnt, h = gpu_run(wasm, "simd", ROWS, [I32], [I64])
    assert compare(ref, rets, st, cnt, h, [I64], exact=True) == []
    ref = oracle_run(m, "lane_oob", OOB_ROWS)
    rets, st, cnt, h = gpu_run(wasm, "lane_oob", OOB_ROWS, [I32, I32], [I32])
    assert compare(ref, rets, st, cnt, h, [I32], exact=True) == []
