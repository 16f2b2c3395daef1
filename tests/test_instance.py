"""Instance semantics: instantiation with a start function, state
that persists across invocations on the same instances (memory, memory size, globals,
dropped data segments) and BatchReset back to a fresh instantiation. Expected values:
the oracle's om_instantiate + repeated om_invoke on one instance (oracle_py.Instance),
which follows lib/executor/instantiate/module.cpp:16-172 and executor.cpp:82-116."""
import pytest

import oracle_py as O
from helpers import compare, emu_run
from wasmedge_amd.wat import assemble

I32 = 0x7F

STATEFUL = assemble(r"""
(module
  (memory 1 4)
  (global $g (mut i32) (i32.const 5))
  (global $h (mut i64) (i64.const 0))
  (data (i32.const 0) "\03\00\00\00")
  (data $p "\aa\bb\cc\dd")
  (func $start
    (global.set $g (i32.add (global.get $g) (i32.load (i32.const 0))))
    (i32.store (i32.const 8) (i32.const 77)))
  (start $start)
  (func (export "step") (param $x i32) (result i32)
    (global.set $g (i32.add (global.get $g) (local.get $x)))
    (i32.store (i32.const 8) (i32.add (i32.load (i32.const 8)) (local.get $x)))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 7)) (i32.const 3))
      (then (drop (memory.grow (i32.const 1)))))
    (if (i32.eq (i32.rem_u (local.get $x) (i32.const 5)) (i32.const 1))
      (then (memory.init $p (i32.const 16) (i32.const 0) (i32.const 4)) (data.drop $p)))
    (if (i32.eq (local.get $x) (i32.const 41)) (then unreachable))
    (global.set $h (i64.add (global.get $h) (i64.extend_i32_u (global.get $g))))
    (i32.add (i32.add (global.get $g) (i32.load (i32.const 8)))
             (i32.add (memory.size) (i32.wrap_i64 (global.get $h))))))
""")

START_TRAPS = assemble(r"""
(module
  (memory 1)
  (func $start (i32.store (i32.const 65534) (i32.const 1)))
  (start $start)
  (func (export "f") (result i32) (i32.const 1)))
""")

ROUNDS = [[[i % 50] for i in range(130)], [[(3 * i + 1) % 50] for i in range(130)],
          [[(7 * i + 2) % 50] for i in range(130)]]


def _oracle_sequence(wasm, rounds, func="step"):
    m = O.Module(wasm)
    insts = [O.Instance(m) for _ in rounds[0]]
    return [[inst.invoke(func, row) for inst, row in zip(insts, rows)] for rows in rounds]


def test_start_function_emulator(built):
    """First invocation after instantiation: the start function has run (globals and
    memory it wrote are visible), its instructions are not counted."""
    ref = _oracle_sequence(STATEFUL, ROUNDS[:1])[0]
    rets, st, cnt, h = emu_run(STATEFUL, "step", ROUNDS[0], [I32], [I32])
    assert compare(ref, rets, st, cnt, h, [I32]) == []


def test_start_trap_oracle():
    m = O.Module(START_TRAPS)
    assert O.Instance(m).error == 0x88


@pytest.mark.gpu
def test_gpu_state_persists_across_runs(built):
    from wasmedge_amd import batch
    ref = _oracle_sequence(STATEFUL, ROUNDS)
    ctx = batch.BatchContext(STATEFUL, len(ROUNDS[0]), device=0)
    try:
        for r, rows in enumerate(ROUNDS):
            rets, st, cnt = ctx.execute("step", batch.make_values(rows, [I32]), 1)
            h = ctx.memory_hash()
            ints = batch.ret_ints(rets)
            got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(rows))]
            assert compare(ref[r], got, st, cnt, h, [I32]) == [], "round %d" % r
        # BatchReset = fresh instantiation: round 0 again gives round 0's answers
        ctx.reset()
        rets, st, cnt = ctx.execute("step", batch.make_values(ROUNDS[0], [I32]), 1)
        ints = batch.ret_ints(rets)
        got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(ROUNDS[0]))]
        assert compare(ref[0], got, st, cnt, ctx.memory_hash(), [I32]) == []
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_start_trap_fails_create(built):
    from wasmedge_amd import batch
    with pytest.raises(batch.WasmEdgeError) as e:
        batch.BatchContext(START_TRAPS, 64, device=0)
    assert e.value.code == 0x88


WRITER = assemble(r"""
(module
  (import "env" "mem_fill" (func $mem_fill (param i32 i32 i32)))
  (memory 2 3)
  (data (i32.const 16) "\11\22\33\44")
  (data $p "\07\07\07\07\07\07")
  ;; poke: old word at a, then a store of each kind at a (selected by k)
  (func (export "poke") (param $a i32) (param $k i32) (result i32)
    (local $old i32)
    (local.set $old (i32.load (local.get $a)))
    (if (i32.eq (local.get $k) (i32.const 0)) (then (i32.store (local.get $a) (i32.const 7))))
    (if (i32.eq (local.get $k) (i32.const 1)) (then (i64.store (local.get $a) (i64.const 0x0707070707070707))))
    (if (i32.eq (local.get $k) (i32.const 2)) (then (i32.store8 (local.get $a) (i32.const 7))))
    (if (i32.eq (local.get $k) (i32.const 3)) (then (v128.store (local.get $a) (v128.const i32x4 7 7 7 7))))
    (if (i32.eq (local.get $k) (i32.const 4)) (then (memory.fill (local.get $a) (i32.const 7) (i32.const 12))))
    (if (i32.eq (local.get $k) (i32.const 5)) (then (memory.copy (local.get $a) (i32.const 16) (i32.const 4))))
    (if (i32.eq (local.get $k) (i32.const 6))
      (then (drop (memory.grow (i32.const 1))) (i32.store (i32.const 131072) (i32.const 9))))
    (if (i32.eq (local.get $k) (i32.const 7)) (then (i32.store16 (local.get $a) (i32.const 0x0707))))
    (if (i32.eq (local.get $k) (i32.const 8))
      (then (v128.store32_lane 2 (local.get $a) (v128.const i32x4 1 2 0x07070707 4))))
    (if (i32.eq (local.get $k) (i32.const 9)) (then (memory.init $p (local.get $a) (i32.const 0) (i32.const 6))))
    (if (i32.eq (local.get $k) (i32.const 10))
      (then (call $mem_fill (local.get $a) (i32.const 9) (i32.const 7))))
    (local.get $old)))
""")


@pytest.mark.gpu
@pytest.mark.parametrize("frames,granule", [("lds", 4), ("vgpr", 4), ("lds", 16), ("vgpr", 128)])
def test_gpu_reset_restores_fresh_memory(built, monkeypatch, frames, granule):
    """BatchReset re-instantiates memory: Reset rewrites only rows below each wave's write
    mark (LS_HWM), so every store kind (scalar, i64, byte, i16, v128, v128 lane, fill,
    copy, memory.init, a host function's write, host SetMemory, stores into grown pages)
    must raise the mark, in both frame kernels (LDS frames and VGPR frames, WB_VFRAME).
    After a Reset each lane reads the fresh image again and the memory hash equals a
    freshly created context's."""
    import hostfuncs
    from wasmedge_amd import batch
    monkeypatch.setenv("WB_VFRAME", "0" if frames == "lds" else "1")
    n = 256
    rows = [[(i * 4093) % (2 * 65536 - 16) & ~15, i % 11] for i in range(n)]
    vals = batch.make_values(rows, [I32, I32])
    ctx = batch.BatchContext(WRITER, n, device=0, memory_granule=granule)
    fresh = batch.BatchContext(WRITER, n, device=0, memory_granule=granule)
    hostfuncs.register(ctx)
    try:
        h0 = fresh.memory_hash()
        r0, st, _ = ctx.execute("poke", vals, 1)
        assert (st == 0).all()
        ctx.set_memory(5, 100000, b"\x01\x02\x03\x04")        # host write, high offset
        r1, st, _ = ctx.execute("poke", vals, 1)              # state persists: sees its writes
        assert (st == 0).all()
        for k in set(range(11)) - {6}:                        # every store kind wrote (6: elsewhere)
            assert any(int(a) != int(b) for i, (a, b) in
                       enumerate(zip(batch.ret_ints(r0)[:, 0], batch.ret_ints(r1)[:, 0]))
                       if rows[i][1] == k), k
        ctx.reset()
        assert list(ctx.memory_hash()) == list(h0)
        assert ctx.memory(5, 100000, 4) == b"\x00" * 4
        r2, st, _ = ctx.execute("poke", vals, 1)              # fresh again: same as the first run
        assert (st == 0).all()
        assert list(batch.ret_ints(r2)[:, 0]) == list(batch.ret_ints(r0)[:, 0])
    finally:
        ctx.close()
        fresh.close()


# an initial memory over 4096 pages puts image rows past 2^26 words,
# whose interleaved index (row * 64) passes 2^32
BIG = assemble(r"""
(module
  (memory 4097 4097)
  (data (i32.const 268435556) "\5a\5b\5c\5d")
  (func (export "touch") (param $x i32) (result i32)
    (local $old i32)
    (local.set $old (i32.load (i32.const 268435556)))
    (i32.store (i32.const 268435556) (local.get $x))
    (i32.store (i32.const 268500000) (local.get $x))
    (local.get $old)))
""")


@pytest.mark.gpu
def test_gpu_reset_memory_over_4096_pages(built):
    from wasmedge_amd import batch
    rows = [[0x11111111 * (i + 1)] for i in range(2)]
    m = O.Module(BIG)
    ref = [m.run("touch", r) for r in rows]
    assert [r[1] for r in ref] == [[0x5D5C5B5A]] * 2
    ctx = batch.BatchContext(BIG, 2, device=0)
    try:
        for _ in range(2):                      # fresh instantiation, then after a Reset
            rets, st, cnt = ctx.execute("touch", batch.make_values(rows, [I32]), 1)
            got = [[int(v)] for v in batch.ret_ints(rets)[:, 0]]
            assert compare(ref, got, st, cnt, ctx.memory_hash(), [I32]) == []
            ctx.reset()
    finally:
        ctx.close()


PEEK = assemble(r"""
(module
  (memory 64)
  (global $g (export "g") (mut i32) (i32.const 5))
  (data (i32.const 1048576) "\01\00\00\00")
  (func (export "peek") (param $a i32) (result i32)
    (i32.add (global.get $g) (i32.add (i32.load (local.get $a)) (i32.load (i32.const 1048576))))))
""")


@pytest.mark.gpu
def test_gpu_host_writes_after_untimed_reset(built):
    """a Reset that does not wait for its init kernels (KernelSeconds
    NULL, no start function) leaves them queued on the context's non-blocking stream;
    host SetMemory / GlobalSetValue right after it must land after them, not be
    overwritten by them (4 MiB of image per lane, so the init kernels take a while)."""
    from wasmedge_amd import batch
    n = 4096
    rows = [[(i * 64) % 4000000 & ~3] for i in range(n)]
    vals = batch.make_values(rows, [I32])
    ctx = batch.BatchContext(PEEK, n, device=0)
    try:
        for rnd in range(3):
            ctx.execute("peek", vals, 1)                 # dirty rows below every write mark
            ctx.reset(timed=False)
            ctx.global_set("g", batch.ALL_INSTANCES, 100 + rnd, I32)
            for i in range(0, n, 97):
                ctx.set_memory(i, rows[i][0], (1000 + i).to_bytes(4, "little"))
            assert ctx.memory_pages(7) == 64
            rets, st, _ = ctx.execute("peek", vals, 1)
            assert (st == 0).all()
            got = batch.ret_ints(rets)[:, 0]
            for i in range(n):
                want = 100 + rnd + 1 + ((1000 + i) if i % 97 == 0 else 0)
                assert int(got[i]) == want, (rnd, i)
    finally:
        ctx.close()
