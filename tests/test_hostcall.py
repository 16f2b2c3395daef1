"""Host-import yield path: lanes that call an imported function park on
the device, the CPU runs the host function per lane (helper.cpp:35-97), and the lanes
resume with its results. Checked against the oracle running the same "env" host module:
returns, ErrCodes (host failure 0x8D, host-side out-of-bounds 0x88, Terminated 0x01 from
exit), reference instruction counts and final-memory hashes."""
import pytest

import oracle_py as O
from helpers import compare, emu_run
from wasmedge_amd.wat import assemble

I32, I64 = 0x7F, 0x7E

HOSTMOD = assemble(r"""
(module
  (import "env" "add_i64" (func $add (param i64 i64) (result i64)))
  (import "env" "mem_sum" (func $sum (param i32 i32) (result i32)))
  (import "env" "mem_fill" (func $fill (param i32 i32 i32)))
  (import "env" "fail" (func $fail (param i32) (result i32)))
  (import "env" "exit" (func $exit (param i32)))
  (import "env" "mix" (func $mix (param i32 f64) (result f64)))
  (type $t2 (func (param i32 i32) (result i32)))
  (memory 1)
  (table 2 funcref)
  (elem (i32.const 0) $sum $local_sum)
  (global $calls (mut i32) (i32.const 0))
  (func $local_sum (param i32 i32) (result i32) (i32.add (local.get 0) (local.get 1)))
  (func $deep (param $x i32) (result i32)
    (global.set $calls (i32.add (global.get $calls) (i32.const 1)))
    (i32.mul (call $sum (local.get $x) (i32.const 8)) (i32.const 3)))
  (func (export "run") (param $iid i32) (result i64)
    (local $i i32) (local $acc i64)
    (loop $l
      (call $fill (i32.mul (local.get $i) (i32.const 16)) (i32.const 16)
                  (i32.add (local.get $iid) (local.get $i)))
      (local.set $acc (call $add (local.get $acc) (i64.extend_i32_u
          (call $sum (i32.const 0) (i32.mul (i32.add (local.get $i) (i32.const 1)) (i32.const 16))))))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $i) (i32.rem_u (local.get $iid) (i32.const 5)))))
    (local.set $acc (i64.add (local.get $acc) (i64.extend_i32_u
      (i32.add (local.get $iid) (call $deep (i32.and (local.get $iid) (i32.const 63)))))))
    (local.set $acc (i64.add (local.get $acc) (i64.extend_i32_u
      (call_indirect (type $t2) (i32.const 3) (local.get $iid) (i32.and (local.get $iid) (i32.const 1))))))
    (local.set $acc (i64.add (local.get $acc)
      (i64.reinterpret_f64 (call $mix (local.get $iid) (f64.const 1.25)))))
    (if (i32.eq (i32.rem_u (local.get $iid) (i32.const 7)) (i32.const 3))
      (then (drop (call $fail (i32.const 1)))))
    (if (i32.eq (i32.rem_u (local.get $iid) (i32.const 11)) (i32.const 4))
      (then (call $exit (i32.const 2))))
    (if (i32.eq (i32.rem_u (local.get $iid) (i32.const 13)) (i32.const 5))
      (then (drop (call $sum (i32.const 65530) (i32.const 100)))))
    (i64.add (local.get $acc) (i64.extend_i32_u (global.get $calls)))))
""")

ROWS = [[i] for i in range(200)]


def test_oracle_host_module():
    m = O.Module(HOSTMOD)
    ref = [m.run("run", r) for r in ROWS]
    codes = {r[0] for r in ref}
    assert codes == {0, 0x01, 0x8D, 0x88}, codes
    assert ref[0][0] == 0 and ref[0][2] > 0


IMPORTS = ["add_i64", "mem_sum", "mem_fill", "fail", "exit", "mix"]


def test_host_calls_emulator_parity(built):
    """The lowering of host calls (direct, nested, via call_indirect) and the result
    placement, on the host emulator with the host functions run inline."""
    from hostfuncs import emu_host
    m = O.Module(HOSTMOD)
    ref = [m.run("run", r) for r in ROWS]
    cb = emu_host(IMPORTS)
    rets, st, cnt, h = emu_run(HOSTMOD, "run", ROWS, [I32], [I64], host=cb)
    assert compare(ref, rets, st, cnt, h, [I64]) == []


@pytest.mark.gpu
def test_gpu_host_calls_parity(built):
    from hostfuncs import register
    from wasmedge_amd import batch
    m = O.Module(HOSTMOD)
    inst = [O.Instance(m) for _ in ROWS]
    ctx = batch.BatchContext(HOSTMOD, len(ROWS), device=0)
    try:
        register(ctx)
        for rnd in range(2):   # state (memory, globals) persists into the second round
            ref = [x.invoke("run", r) for x, r in zip(inst, ROWS)]
            rets, st, cnt = ctx.execute("run", batch.make_values(ROWS, [I32]), 1)
            ints = batch.ret_ints(rets)
            got = [[int(v) for v in ints[i]] if st[i] == 0 else [] for i in range(len(ROWS))]
            assert compare(ref, got, st, cnt, ctx.memory_hash(), [I64]) == [], rnd
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_unregistered_import_status(built):
    from wasmedge_amd import batch
    ctx = batch.BatchContext(HOSTMOD, 64, device=0)
    try:
        rets, st, cnt = ctx.execute("run", batch.make_values([[i] for i in range(64)], [I32]), 1)
        assert all(int(s) == 0xB1 for s in st)
    finally:
        ctx.close()


SERIAL = assemble(r"""
(module
  (import "env" "tick" (func $tick (param i32) (result i32)))
  (func (export "run") (param $iid i32) (result i32)
    (call $tick (local.get $iid))))
""")


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [0, 1])
def test_gpu_default_host_threads_are_serial(built, threads):
    """HostThreads 0 (the default) and 1 call host functions one at a time from one
    thread, so a host function with shared mutable state (a plain counter, no lock) is
    safe there; only HostThreads > 1 asks for reentrant host functions."""
    import threading
    import time
    from wasmedge_amd import batch
    n = 640   # 10 waves
    state = {"inside": 0, "overlap": 0, "count": 0, "tids": set()}

    def tick(mem, a):
        state["inside"] += 1
        if state["inside"] > 1:
            state["overlap"] += 1
        state["tids"].add(threading.get_ident())
        c = state["count"]
        time.sleep(0)        # would let a second service thread in
        state["count"] = c + 1
        state["inside"] -= 1
        return 0, [(a[0] * 3 + 1) & 0xFFFFFFFF]

    ctx = batch.BatchContext(SERIAL, n, device=0, host_threads=threads)
    try:
        ctx.add_host_function("env", "tick", tick, 1, 1)
        rets, st, cnt = ctx.execute("run", batch.make_values([[i] for i in range(n)], [I32]), 1)
        assert all(int(s) == 0 for s in st)
        assert [int(v[0]) for v in batch.ret_ints(rets)] == [(3 * i + 1) & 0xFFFFFFFF for i in range(n)]
        assert state["count"] == n and state["overlap"] == 0 and len(state["tids"]) == 1
    finally:
        ctx.close()
