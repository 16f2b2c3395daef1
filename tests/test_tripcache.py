"""Trip mode's same-trip shortcuts (jit.cpp trip_source), against the oracle:

- the load cache: a scan that ends leaves the word it ended on (and its address) in VGPRs;
  a later run whose loads are all at such addresses runs in the same trip (LtF);
- the successor-window prefetch: a scan that falls into another scan loads the second
  scan's window too; lanes that leave the first scan run the second in the same trip (LtS);
- br_table threading: a jump onto a run that is one br_table (a state machine's dispatch)
  takes the table itself, so a state whose successor lies ahead runs in the same trip.

Both are only right while no store of the lane has touched the cached words: the module
below stores into the prefetched window (run X, which also jumps past the first scan
straight into the second) and onto the cached word (the `if` before the consumer), and
every result, status, instruction count and memory image must still equal the oracle's,
with either shortcut on or off (WB_TRIP_PF, WB_TRIP_FWD; trip mode forced, WB_TRIP=1).
"""
import ctypes
import os

import pytest

import oracle_py as O
from helpers import compare
from wasmedge_amd import workloads as W
from wasmedge_amd.wat import assemble

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
I32 = 0x7F

SCANS_WAT = r"""
(module
  (memory 1)
  (func (export "run") (param $seed i32) (param $n i32) (result i32)
    (local $x i32) (local $k i32) (local $i i32) (local $j i32) (local $p i32)
    (local $c i32) (local $sum i32) (local $end i32)
    (local.set $x (i32.or (i32.mul (local.get $seed) (i32.const 2654435761)) (i32.const 1)))
    (local.set $end (i32.add (i32.const 68) (i32.shl (local.get $n) (i32.const 2))))
    (i32.store (i32.const 64) (i32.const 0x80000000))
    (local.set $k (i32.const 68))
    (block $filled
      (loop $fill
        (br_if $filled (i32.ge_u (local.get $k) (local.get $end)))
        (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 13))))
        (local.set $x (i32.xor (local.get $x) (i32.shr_u (local.get $x) (i32.const 17))))
        (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 5))))
        (i32.store (local.get $k) (i32.shr_s (local.get $x) (i32.const 26)))
        (local.set $k (i32.add (local.get $k) (i32.const 4)))
        (br $fill)))
    (i32.store (local.get $end) (i32.const 0x7fffffff))
    (local.set $p (i32.shr_s (i32.mul (local.get $seed) (i32.const 0x9e3779b1)) (i32.const 28)))
    (local.set $i (i32.const 64))
    (local.set $j (local.get $end))
    (loop $outer
      (block $toj
        ;; run X: a store into the window the first scan prefetched for the second; every
        ;; other round straight on to the second scan
        (i32.store (i32.sub (local.get $j) (i32.const 4))
          (i32.add (local.get $p) (i32.sub (i32.rem_u (local.get $c) (i32.const 3)) (i32.const 1))))
        (br_if $toj (i32.and (local.get $c) (i32.const 1)))
        (loop $li
          (local.set $i (i32.add (local.get $i) (i32.const 4)))
          (br_if $li (i32.lt_s (i32.load (local.get $i)) (local.get $p)))))
      (loop $lj
        (local.set $j (i32.sub (local.get $j) (i32.const 4)))
        (br_if $lj (i32.gt_s (i32.load (local.get $j)) (local.get $p))))
      ;; a store onto the word the second scan ended on, before its consumer
      (if (i32.and (local.get $c) (i32.const 2))
        (then (i32.store (local.get $j) (i32.add (local.get $c) (i32.const 1000)))))
      (local.set $sum (i32.add (i32.mul (local.get $sum) (i32.const 31))
        (i32.add (i32.load (local.get $i)) (i32.load (local.get $j)))))
      (local.set $c (i32.add (local.get $c) (i32.const 1)))
      (br_if $outer (i32.lt_u (local.get $c) (i32.const 12))))
    (i32.add (local.get $sum) (i32.add (local.get $i) (i32.shl (local.get $j) (i32.const 16)))))
)
"""


# a br_table state machine (C4's shape) whose states jump back to the dispatch with the
# next state set to a constant (in range, and past the table: its default entry) or computed
MACHINE_WAT = r"""
(module
  (memory 1)
  (func (export "run") (param $seed i32) (param $n i32) (result i32)
    (local $x i32) (local $state i32) (local $k i32) (local $acc i32)
    (local.set $x (i32.or (i32.mul (local.get $seed) (i32.const 2654435761)) (i32.const 1)))
    (block $done
      (loop $machine
        (block $s3
          (block $s2
            (block $s1
              (block $s0
                (br_table $s0 $s1 $s2 $s3 (local.get $state)))
              ;; 0: step the generator; computed next state (0..5: 4 and 5 take the default)
              (br_if $done (i32.ge_u (local.get $k) (local.get $n)))
              (local.set $k (i32.add (local.get $k) (i32.const 1)))
              (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 13))))
              (local.set $x (i32.xor (local.get $x) (i32.shr_u (local.get $x) (i32.const 17))))
              (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 5))))
              (local.set $state (i32.rem_u (local.get $x) (i32.const 6)))
              (br $machine))
            ;; 1: constant next state 0
            (local.set $acc (i32.add (local.get $acc) (local.get $x)))
            (local.set $state (i32.const 0))
            (br $machine))
          ;; 2: constant next state past the table (the default: 3)
          (local.set $acc (i32.xor (local.get $acc) (i32.mul (local.get $x) (i32.const 3))))
          (local.set $state (i32.const 9))
          (br $machine))
        ;; 3 (and the default): a store, then state 1 or 0 by a parity
        (i32.store (i32.and (local.get $x) (i32.const 1020)) (local.get $acc))
        (local.set $state (i32.and (local.get $acc) (i32.const 1)))
        (br $machine)))
    (i32.add (local.get $acc) (i32.load (i32.const 64))))
)
"""


def machine_wasm():
    return assemble(MACHINE_WAT)


def scans_wasm():
    return assemble(SCANS_WAT)


def rows():
    return [[s, n] for s in range(256) for n in (0, 1, 2, 5, 9, 16, 33, 60)]


def _trip_dump(wasm, tmp_path, monkeypatch):
    L = ctypes.CDLL(os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch.so"))
    L.wb_jit_check.restype = ctypes.c_int
    L.wb_jit_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_uint32]
    dump = tmp_path / "trip.s"
    monkeypatch.setenv("WB_JIT_DUMP_TRIP", str(dump))
    err = ctypes.create_string_buffer(4096)
    ins = ctypes.c_uint32(0)
    assert L.wb_jit_check(wasm, len(wasm), 7, ctypes.byref(ins), err, 4096) > 0, err.value
    return dump.read_text()


def test_module_runs_on_oracle():
    """the module ends both ways (results and traps) over the rows"""
    m = O.Module(scans_wasm())
    codes = {m.run("run", r)[0] for r in rows()[::7]}
    assert 0 in codes and len(codes) >= 2


@pytest.mark.parametrize("name", ["c3", "scans"])
def test_trip_code_has_both_shortcuts(built, tmp_path, monkeypatch, name):
    """C3 and the test module compile a prefetched second scan (LtS) and a consumer of the
    cached words (LtF); WB_TRIP_PF=0 / WB_TRIP_FWD=0 drop them."""
    wasm = W.qsort_wasm() if name == "c3" else scans_wasm()
    src = _trip_dump(wasm, tmp_path, monkeypatch)
    assert "LtS" in src and "LtF" in src and "_pf:" in src
    monkeypatch.setenv("WB_TRIP_PF", "0")
    monkeypatch.setenv("WB_TRIP_FWD", "0")
    src = _trip_dump(wasm, tmp_path, monkeypatch)
    assert "LtS" not in src and "LtF" not in src


@pytest.mark.gpu
@pytest.mark.parametrize("pf,fwd", [("1", "1"), ("0", "1"), ("1", "0")])
def test_gpu_shortcuts_exact(built, monkeypatch, pf, fwd):
    monkeypatch.setenv("WB_TRIP", "1")
    monkeypatch.setenv("WB_TRIP_PF", pf)
    monkeypatch.setenv("WB_TRIP_FWD", fwd)
    from wasmedge_amd import batch
    wasm = scans_wasm()
    rs = rows()
    m = O.Module(wasm)
    ref = [m.run("run", r) for r in rs]
    ctx = batch.BatchContext(wasm, len(rs))
    try:
        assert ctx.compiled_runs() > 0
        rets, st, cnt = ctx.execute("run", batch.make_values(rs, [I32, I32]), 1)
        h = ctx.memory_hash()
        ints = batch.ret_ints(rets)
    finally:
        ctx.close()
    got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(rs))]
    assert compare(ref, got, st, cnt, h, [I32], exact=True) == []


def test_machine_threads_its_dispatch(built, tmp_path, monkeypatch):
    """the state runs' jumps take the br_table themselves: a state with a computed next
    state carries a copy of the table's compare chain (v_min_u32 clamps its index), one
    with a constant next state jumps straight on; WB_BRT_THREAD=0 leaves the dispatch run's
    chain alone"""
    for wasm, copies in ((W.collatz_wasm(), 1), (machine_wasm(), 2)):
        on = _trip_dump(wasm, tmp_path, monkeypatch).count("v_min_u32")
        monkeypatch.setenv("WB_BRT_THREAD", "0")
        off = _trip_dump(wasm, tmp_path, monkeypatch).count("v_min_u32")
        monkeypatch.delenv("WB_BRT_THREAD")
        assert on - off == copies
    m = O.Module(machine_wasm())
    assert {m.run("run", r)[0] for r in rows()[:64]} == {0}


@pytest.mark.gpu
@pytest.mark.parametrize("thread", ["1", "0"])
def test_gpu_machine_exact(built, monkeypatch, thread):
    monkeypatch.setenv("WB_TRIP", "1")
    monkeypatch.setenv("WB_BRT_THREAD", thread)
    from wasmedge_amd import batch
    wasm = machine_wasm()
    rs = [[s, n] for s in range(512) for n in (0, 1, 7, 40, 300)]
    m = O.Module(wasm)
    ref = [m.run("run", r) for r in rs]
    ctx = batch.BatchContext(wasm, len(rs))
    try:
        assert ctx.compiled_runs() > 0
        rets, st, cnt = ctx.execute("run", batch.make_values(rs, [I32, I32]), 1)
        h = ctx.memory_hash()
        ints = batch.ret_ints(rets)
    finally:
        ctx.close()
    got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(rs))]
    assert compare(ref, got, st, cnt, h, [I32], exact=True) == []


@pytest.mark.gpu
@pytest.mark.parametrize("pf,fwd", [("1", "1"), ("0", "0")])
def test_gpu_c3_shortcuts_exact(built, monkeypatch, pf, fwd):
    """C3 at 300 elements (scans of every length, partitions down to one element)"""
    monkeypatch.setenv("WB_TRIP_PF", pf)
    monkeypatch.setenv("WB_TRIP_FWD", fwd)
    from wasmedge_amd import batch
    wasm = W.qsort_wasm()
    rs = [[i, 300] for i in range(1024)]
    m = O.Module(wasm)
    ref = [m.run("sort", r) for r in rs[:96]]
    ctx = batch.BatchContext(wasm, len(rs))
    try:
        rets, st, cnt = ctx.execute("sort", batch.make_values(rs, [I32, I32]), 1)
        h = ctx.memory_hash()
        ints = batch.ret_ints(rets)
    finally:
        ctx.close()
    got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(96)]
    assert compare(ref, got, st[:96], cnt[:96], h[:96], [I32], exact=True) == []
