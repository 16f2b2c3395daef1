"""Compiled accesses to memories past the first (MultiMemories).

XLD / XST -- a load or store on memory k >= 1 -- compile into the runs (jit.cpp emit_xmem):
the lane's word w of memory k is at the wave's block (s[98:99], set by the kernel at every
core call) + (xinfo[2 (k - 1)] + w) * 256 + lane * 4, checked against the module's declared
minimum size of memory k; a misaligned access, one past that minimum (a grown memory's new
pages) and an out-of-bounds one leave before the instruction and the C++ step executes it
(dbc_step.inc OP_XLD / OP_XST, memory.ipp:12-68 on getMemInstByIdx's memory). The GPU tests
compare every lane with the oracle's restatement on the compiled runs (SIMT and trip mode)
and on the threaded core alone (WB_JIT=0); the results fold in memories 1 and 2 (the memory
hash covers memory 0)."""
import ctypes
import os

import pytest

import oracle_py as O
from helpers import compare, emu_run
from wasmedge_amd.wat import assemble
from wasmedge_amd import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
I32 = 0x7F

# every load and store width on memories 1 (1 page, max 4) and 2 (2 pages), sub-word
# accesses at any byte, an offset past the 4 KiB instruction field (70000 * 64), v128,
# misaligned words, memory 1 grown past its minimum for seed % 3 == 0 (its accesses then
# reach the grown page), and a trap past memory 1's end for seed % 13 == 0
XJ_WAT = r"""
(module
  (memory $m0 1)
  (memory $m1 1 4)
  (memory $m2 2)
  (data (memory $m2) (i32.const 8) "second memory")
  (func (export "run") (param $seed i32) (param $n i32) (result i32)
    (local $k i32) (local $acc i32) (local $x i32) (local $mask i32) (local $a i32)
    (local.set $x (i32.or (i32.mul (local.get $seed) (i32.const 2654435761)) (i32.const 1)))
    (local.set $mask (i32.const 0xfffc))
    (if (i32.eqz (i32.rem_u (local.get $seed) (i32.const 3)))
      (then (drop (memory.grow $m1 (i32.const 1)))
            (local.set $mask (i32.const 0x1fffc))))
    (block $done
      (loop $l
        (br_if $done (i32.ge_u (local.get $k) (local.get $n)))
        (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 13))))
        (local.set $x (i32.xor (local.get $x) (i32.shr_u (local.get $x) (i32.const 17))))
        (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 5))))
        (local.set $a (i32.and (local.get $x) (local.get $mask)))
        (i32.store $m1 (local.get $a) (local.get $x))
        (i32.store8 $m1 offset=3 (i32.and (i32.shr_u (local.get $x) (i32.const 8)) (i32.const 0xfff0))
                    (local.get $k))
        (i32.store16 $m2 offset=70000 (i32.and (i32.shr_u (local.get $x) (i32.const 3)) (i32.const 0x7ffe))
                     (local.get $x))
        (i64.store $m2 (i32.and (i32.shr_u (local.get $x) (i32.const 5)) (i32.const 0x1fff8))
                   (i64.or (i64.shl (i64.extend_i32_u (local.get $k)) (i64.const 32))
                           (i64.extend_i32_u (local.get $x))))
        (i64.store32 $m1 offset=8 (i32.and (local.get $x) (i32.const 0x3ff8)) (i64.extend_i32_s (local.get $acc)))
        (local.set $acc (i32.add (local.get $acc)
          (i32.load8_s $m1 (i32.and (local.get $x) (i32.const 0xffff)))))
        (local.set $acc (i32.xor (local.get $acc)
          (i32.load8_u $m2 offset=1 (i32.and (i32.shr_u (local.get $x) (i32.const 9)) (i32.const 0x1fffe)))))
        (local.set $acc (i32.add (local.get $acc)
          (i32.load16_s $m1 (i32.and (local.get $x) (i32.const 0xfffe)))))
        (local.set $acc (i32.xor (local.get $acc)
          (i32.load16_u $m2 offset=70000 (i32.and (i32.shr_u (local.get $x) (i32.const 11)) (i32.const 0x7ffe)))))
        (local.set $acc (i32.add (local.get $acc)
          (i32.wrap_i64 (i64.load $m2 (i32.and (i32.shr_u (local.get $x) (i32.const 7)) (i32.const 0x1fff8))))))
        (local.set $acc (i32.add (local.get $acc)
          (i32.wrap_i64 (i64.shr_u (i64.load $m2 (i32.and (local.get $x) (i32.const 0x1fff8))) (i64.const 32)))))
        (local.set $acc (i32.xor (local.get $acc)
          (i32.wrap_i64 (i64.shr_s (i64.load32_s $m1 (local.get $a)) (i64.const 7)))))
        (local.set $acc (i32.add (local.get $acc)
          (i32.wrap_i64 (i64.shr_u (i64.load32_u $m1 (local.get $a)) (i64.const 3)))))
        (local.set $acc (i32.add (local.get $acc)
          (i32.wrap_i64 (i64.shr_s (i64.load8_s $m1 offset=2 (local.get $a)) (i64.const 40)))))
        (local.set $acc (i32.add (local.get $acc)
          (i32.wrap_i64 (i64.load16_u $m2 offset=6 (i32.and (local.get $x) (i32.const 0xfffe))))))
        (local.set $acc (i32.xor (local.get $acc)
          (i32.wrap_i64 (i64.shr_s (i64.load16_s $m1 (i32.and (local.get $x) (i32.const 0xfffe))) (i64.const 48)))))
        (local.set $acc (i32.add (local.get $acc)
          (i32.wrap_i64 (i64.load8_u $m2 (i32.and (local.get $x) (i32.const 0x1ffff))))))
        ;; 8 and 16 bytes at 4 mod 8 / 4 mod 16 (across granules of 8 or 16 bytes)
        (local.set $acc (i32.xor (local.get $acc)
          (i32.wrap_i64 (i64.shr_u (i64.load $m2 offset=4 (i32.and (local.get $x) (i32.const 0xfff0))) (i64.const 16)))))
        (local.set $acc (i32.add (local.get $acc)
          (i32x4.extract_lane 2 (v128.load $m1 offset=4 (i32.and (i32.shr_u (local.get $x) (i32.const 2)) (i32.const 0xffe0))))))
        (i64.store $m1 offset=12 (i32.and (i32.shr_u (local.get $x) (i32.const 6)) (i32.const 0xfff0)) (i64.extend_i32_u (local.get $acc)))
        ;; a misaligned word (lanes leave to the per-lane step) every 4th trip
        (if (i32.eqz (i32.and (local.get $k) (i32.const 3)))
          (then (local.set $acc (i32.add (local.get $acc)
                  (i32.load $m1 offset=1 (i32.and (local.get $x) (i32.const 0xfff8)))))))
        (v128.store $m2 offset=16 (i32.and (local.get $x) (i32.const 0xfff0))
                    (i32x4.splat (i32.add (local.get $x) (local.get $k))))
        (local.set $acc (i32.add (local.get $acc)
          (i32x4.extract_lane 3 (v128.load $m1 (i32.and (local.get $x) (i32.const 0xfff0))))))
        (local.set $acc (i32.xor (local.get $acc)
          (i32x4.extract_lane 1 (v128.load $m2 offset=16 (i32.and (i32.shr_u (local.get $x) (i32.const 4)) (i32.const 0xfff0))))))
        (i32.store $m0 (i32.shl (i32.and (local.get $k) (i32.const 63)) (i32.const 2)) (local.get $acc))
        (local.set $k (i32.add (local.get $k) (i32.const 1)))
        (br $l)))
    ;; fold the first 1 KiB of memories 1 and 2 into the result
    (local.set $k (i32.const 0))
    (block $sd
      (loop $s
        (br_if $sd (i32.ge_u (local.get $k) (i32.const 1024)))
        (local.set $acc (i32.add (i32.mul (local.get $acc) (i32.const 31))
          (i32.xor (i32.load $m1 (local.get $k)) (i32.load $m2 offset=70000 (local.get $k)))))
        (local.set $k (i32.add (local.get $k) (i32.const 4)))
        (br $s)))
    (if (i32.eqz (i32.rem_u (local.get $seed) (i32.const 13)))
      (then (drop (i32.load $m1 (i32.sub (i32.shl (memory.size $m1) (i32.const 16)) (i32.const 2))))))
    (local.get $acc))
)
"""


def xj_wasm():
    return assemble(XJ_WAT)


def rows():
    return [[s, n] for s in range(256) for n in (0, 3, 40, 150)]


def _check_lib():
    L = ctypes.CDLL(os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch.so"))
    L.wb_jit_check.restype = ctypes.c_int
    L.wb_jit_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_uint32]
    return L


def test_module_runs_on_oracle():
    """the rows end both ways: results, and the trap past memory 1"""
    m = O.Module(xj_wasm(), multi_memory=True)
    out = [m.run("run", r) for r in rows()[::5]]
    assert {o[0] for o in out} == {0, 0x88}
    assert len({o[1][0] for o in out if o[0] == 0}) > 30


def test_emulator_matches_oracle(built):
    wasm = xj_wasm()
    rs = rows()[::3]
    ref = [O.Module(wasm, multi_memory=True).run("run", r) for r in rs]
    got = emu_run(wasm, "run", rs, [I32, I32], [I32], multi_memory=True)
    assert compare(ref, *got, [I32], exact=True) == []


@pytest.mark.parametrize("name", ["xj", "c3x"])
def test_accesses_compile(built, tmp_path, monkeypatch, name):
    """every flavour of the compiled runs (plain, SIMT, trip) compiles the extra-memory
    accesses: their code addresses the wave's block through s[98:99]"""
    wasm = xj_wasm() if name == "xj" else W.qsort_x_wasm()
    for k in ("", "_SIMT", "_TRIP"):
        monkeypatch.setenv("WB_JIT_DUMP" + k, str(tmp_path / ("d%s.s" % k)))
    err = ctypes.create_string_buffer(4096)
    n = ctypes.c_uint32()
    assert _check_lib().wb_jit_check(wasm, len(wasm), 0, ctypes.byref(n), err, 4096) > 0, err.value
    for k in ("", "_SIMT", "_TRIP"):
        assert "s[98:99]" in (tmp_path / ("d%s.s" % k)).read_text(), k


def _gpu_rows(wasm, func, rs, env, monkeypatch, reps=2):
    from wasmedge_amd import batch
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ctx = batch.BatchContext(wasm, len(rs), multi_memory=True)
    out = []
    try:
        for rep in range(reps):
            if rep:
                ctx.reset()
            rets, st, cnt = ctx.execute(func, batch.make_values(rs, [I32, I32]), 1)
            ints = batch.ret_ints(rets)
            got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(rs))]
            out.append((got, st, cnt, ctx.memory_hash()))
        runs = ctx.compiled_runs()
    finally:
        ctx.close()
    return out, runs


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{}, {"WB_TRIP": "0"}, {"WB_TRIP": "1"}, {"WB_JIT": "0"},
                                 {"WB_XGRAN": "4"}, {"WB_XGRAN": "8"}, {"WB_XGRAN": "16"},
                                 {"WB_XGRAN": "4", "WB_JIT": "0"}],
                         ids=["default", "simt", "trip", "core", "gran4", "gran8", "gran16", "gran4-core"])
def test_gpu_extra_memory_accesses(built, monkeypatch, env):
    """bit-exact against the oracle on every engine and granule of the extra memories
    (the default for this module's data-dependent addresses: 128 bytes), twice around a
    Reset"""
    wasm = xj_wasm()
    rs = rows()
    ref = [O.Module(wasm, multi_memory=True).run("run", r) for r in rs]
    assert {r[0] for r in ref} == {0, 0x88}
    out, runs = _gpu_rows(wasm, "run", rs, env, monkeypatch)
    assert (runs > 0) == (env.get("WB_JIT") != "0")
    for rets, st, cnt, h in out:
        assert compare(ref, rets, st, cnt, h, [I32], exact=True) == []


def scans_x_wasm():
    """tests/test_tripcache.py's scan module (stores into a prefetched window and onto a
    cached word) with its memory as memory 1: trip mode's scan windows, successor-window
    prefetch and load cache on an extra memory"""
    from test_tripcache import SCANS_WAT
    src = SCANS_WAT.replace("  (memory 1)", "  (memory $m0 1)\n  (memory $m1 1)")
    for op in ("i32.load", "i32.store"):
        src = src.replace("(%s " % op, "(%s $m1 " % op)
    return assemble(src)


def test_scan_module_on_oracle():
    from test_tripcache import rows as scan_rows, scans_wasm
    m, m0 = O.Module(scans_x_wasm(), multi_memory=True), O.Module(scans_wasm())
    for r in scan_rows()[::17]:
        a, b = m.run("run", r), m0.run("run", r)
        assert a[:3] == b[:3]


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"WB_TRIP": "1"}, {"WB_TRIP": "1", "WB_TRIP_PF": "0"},
                                 {"WB_TRIP": "1", "WB_TRIP_FWD": "0"}, {"WB_TRIP": "1", "WB_TRIP_SCAN": "0"}],
                         ids=["trip", "no-pf", "no-fwd", "no-scan"])
def test_gpu_scans_on_memory_1(built, monkeypatch, env):
    from test_tripcache import rows as scan_rows
    wasm = scans_x_wasm()
    rs = scan_rows()
    ref = [O.Module(wasm, multi_memory=True).run("run", r) for r in rs]
    out, runs = _gpu_rows(wasm, "run", rs, env, monkeypatch)
    assert runs > 0
    for rets, st, cnt, h in out:
        assert compare(ref, rets, st, cnt, h, [I32], exact=True) == []


@pytest.mark.gpu
def test_gpu_c3_on_memory_1(built, monkeypatch):
    """C3's quicksort on memory 1 (bench.py --workload c3x) at 4096 instances x 2000
    elements: every lane's result and count equal C3's on memory 0 (GPU), and a sample the
    oracle's"""
    wasm = W.qsort_x_wasm()
    rs = [[i, 2000] for i in range(4096)]
    m = O.Module(wasm, multi_memory=True)
    ref = [m.run("sort", r) for r in rs[::37]]
    out, runs = _gpu_rows(wasm, "sort", rs, {}, monkeypatch, reps=1)
    assert runs > 0
    rets, st, cnt, _ = out[0]
    assert (st == 0).all()
    got = [(0, [rets[i][0] & 0xFFFFFFFF], int(cnt[i])) for i in range(0, 4096, 37)]
    assert got == [(r[0], [r[1][0] & 0xFFFFFFFF], r[2]) for r in ref]
    from wasmedge_amd import batch
    ctx = batch.BatchContext(W.qsort_wasm(), len(rs))
    try:
        rets0, st0, cnt0 = ctx.execute("sort", batch.make_values(rs, [I32, I32]), 1)
        ints0 = batch.ret_ints(rets0)
    finally:
        ctx.close()
    assert (st0 == 0).all() and (cnt0 == cnt).all()
    assert [int(ints0[i][0]) & 0xFFFFFFFF for i in range(len(rs))] == [r[0] & 0xFFFFFFFF for r in rets]


@pytest.mark.gpu
@pytest.mark.parametrize("gran", ["4", "16", "128"])
def test_gpu_bulk_ops_by_granule(built, monkeypatch, gran):
    """tests/test_multimem.py's module (size / grow / fill / init / copy within and across
    memories, v128 and lane forms, an active data segment on memory 1, traps on memories
    1 and 2) with the extra memories in granules of 4, 16 and 128 bytes"""
    from test_multimem import mm_wasm, rows as mm_rows
    wasm = mm_wasm()
    rs = mm_rows()
    ref = [O.Module(wasm, multi_memory=True).run("run", r) for r in rs]
    out, _ = _gpu_rows(wasm, "run", rs, {"WB_XGRAN": gran}, monkeypatch)
    for rets, st, cnt, h in out:
        assert compare(ref, rets, st, cnt, h, [I32], exact=True) == []
