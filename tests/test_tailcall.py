"""Tail calls (the TailCall proposal: return_call, return_call_indirect; opt-in in the
reference, configure.h:176-182). The reference enters the callee with IsTailCall
(controlInstr.cpp:83-158, helper.cpp:16-177): the caller's frame is reused
(stackmgr.h:85-97), so the callee returns straight to the caller's caller and the stack does
not grow. Here a TAIL_CALL moves the arguments to the frame base and jumps, pushing no
return record (dbc_step.inc). Checked against the oracle's restatement (oracle/
wasm_oracle_exec.inc tail_frame); the reference holds no tail-call fixture (its spec corpus
is fetched at build time), so beyond the oracle the counts are parity
unpinned. Results are pinned independently by each module's non-tail twin."""
import pytest

import oracle_py as O
from helpers import compare, emu_run, gpu_run
from wasmedge_amd.wat import assemble

I32, I64 = 0x7F, 0x7E


def tail_wat(call):
    """`call` = "return_call" or, for the twin, "call" (same results, a growing stack)."""
    return r"""
(module
  (type $t2 (func (param i64 i64) (result i64)))
  (table 4 funcref)
  (elem (i32.const 0) $sum $even $odd $mix)
  (memory 1)
  ;; sum 1..n by tail recursion
  (func $sum (param $n i64) (param $acc i64) (result i64)
    (if (result i64) (i64.eqz (local.get $n))
      (then (local.get $acc))
      (else (%(c)s $sum (i64.sub (local.get $n) (i64.const 1))
                         (i64.add (local.get $acc) (local.get $n))))))
  ;; mutual recursion, with locals the tail call must zero
  (func $even (param $n i64) (param $k i64) (result i64) (local $z i64)
    (local.set $z (i64.add (local.get $z) (i64.const 3)))
    (if (result i64) (i64.eqz (local.get $n))
      (then (i64.add (local.get $k) (local.get $z)))
      (else (%(c)s $odd (i64.sub (local.get $n) (i64.const 1)) (i64.add (local.get $k) (local.get $z))))))
  (func $odd (param $n i64) (param $k i64) (result i64) (local $y i32)
    (local.set $y (i32.add (local.get $y) (i32.const 1)))
    (i32.store (i32.wrap_i64 (i64.and (local.get $n) (i64.const 1020))) (local.get $y))
    (if (result i64) (i64.eqz (local.get $n))
      (then (i64.sub (local.get $k) (i64.extend_i32_u (local.get $y))))
      (else (%(c)s $even (i64.sub (local.get $n) (i64.const 1)) (i64.mul (local.get $k) (i64.const 3))))))
  ;; through the table: the callee picked by n
  (func $mix (param $n i64) (param $k i64) (result i64)
    (if (result i64) (i64.le_u (local.get $n) (i64.const 1))
      (then (local.get $k))
      (else (%(c)s_indirect (type $t2) (i64.sub (local.get $n) (i64.const 1))
                                   (i64.xor (local.get $k) (local.get $n))
                                   (i32.wrap_i64 (i64.rem_u (local.get $n) (i64.const 4)))))))
  (func (export "run") (param $which i32) (param $n i32) (result i64)
    (local $nn i64)
    (local.set $nn (i64.extend_i32_u (local.get $n)))
    (if (result i64) (i32.eq (local.get $which) (i32.const 0))
      (then (call $sum (local.get $nn) (i64.const 0)))
      (else (if (result i64) (i32.eq (local.get $which) (i32.const 1))
        (then (call $even (local.get $nn) (i64.const 7)))
        (else (i64.add (i64.const 1) (call $mix (local.get $nn) (i64.const 5))))))))
  ;; the entry function itself tail-calls
  (func (export "direct") (param $n i32) (result i64)
    (%(c)s $sum (i64.extend_i32_u (local.get $n)) (i64.const 100)))
)
""" % {"c": call}


TAIL = assemble(tail_wat("return_call"))
TWIN = assemble(tail_wat("call"))
ROWS = [[w, n] for w in range(3) for n in (0, 1, 2, 3, 7, 64, 300, 1001)]


def test_oracle_gate_and_twin():
    """Off by default (IllegalOpCode 0x37, loader/ast/instruction.cpp:903-907); on, every
    result equals the non-tail twin's, and the tail version retires fewer instructions
    (no caller continuation after each call)."""
    with pytest.raises(O.OracleError) as e:
        O.Module(TAIL)
    assert "0x37" in str(e.value)
    m, t = O.Module(TAIL, tail_call=True), O.Module(TWIN)
    for row in ROWS:
        a, b = m.run("run", row), t.run("run", row)
        assert a[0] == b[0] == 0 and a[1] == b[1], row
        assert a[2] < b[2] or row[1] == 0 or (row[0] == 2 and row[1] <= 1), row
    assert m.run("direct", [10]) [1] == [155]


def test_emulator_matches_oracle(built):
    m = O.Module(TAIL, tail_call=True)
    for func, rows, pt in (("run", ROWS, [I32, I32]), ("direct", [[n] for n in (0, 5, 999)], [I32])):
        ref = [m.run(func, r) for r in rows]
        assert compare(ref, *emu_run(TAIL, func, rows, pt, [I64], tail_call=True), [I64]) == []


def test_emulator_gate(built):
    with pytest.raises(RuntimeError, match="0x37"):
        emu_run(TAIL, "run", [[0, 1]], [I32, I32], [I64])


INDIRECT_TRAPS = assemble(r"""
(module
  (type $t (func (param i32) (result i32)))
  (type $u (func (param i32 i32) (result i32)))
  (import "env" "fail" (func $hostf (param i32) (result i32)))
  (table 5 funcref)
  (elem (i32.const 0) $inc $two $hostf)
  (func $inc (param i32) (result i32) (i32.add (local.get 0) (i32.const 1)))
  (func $two (param i32 i32) (result i32) (local.get 0))
  (func (export "go") (param $i i32) (result i32)
    (return_call_indirect (type $t) (i32.const 41) (local.get $i))))
""")


def test_indirect_traps_emulator(built):
    """Index 0 runs; 1: IndirectCallTypeMismatch 0x8C; 3: UninitializedElement 0x8A;
    5: UndefinedElement 0x8B (controlInstr.cpp:101-158, the oracle's order); 2: the host
    import "fail" through the tail call, which fails (41 != 0): ExecutionFailed 0x8D."""
    rows = [[0], [1], [3], [5], [2]]
    m = O.Module(INDIRECT_TRAPS, tail_call=True)
    ref = [m.run("go", r) for r in rows]
    assert [r[0] for r in ref] == [0, 0x8C, 0x8A, 0x8B, 0x8D] and ref[0][1] == [42]
    from hostfuncs import emu_host
    rets, st, cnt, h = emu_run(INDIRECT_TRAPS, "go", rows, [I32], [I32], tail_call=True,
                               host=emu_host(["fail"]))
    assert compare(ref, rets, st, cnt, h, [I32]) == []


# Host imports in tail position (helper.cpp:35-97 with IsTailCall): the host function runs
# in the reused frame and pops it. From the entry function (go, go_ind) the reference then
# re-executes the entry's final `end` (the frame's From is RetIt - 1, helper.cpp:163) and
# returns the host's results: the oracle restates it, the batched path matches it (one
# counted `end` after the host call). From a nested frame (outer -> mid -> return_call) the
# reference re-executes outer's `call` instead (the same off-by-one); the batched path
# returns to outer, as `call $f` + `return` would (HOST_TWIN, which also counts the same two
# instructions), a deliberate divergence (DESIGN.md "Tail calls").
HOST_TAIL_WAT = r"""
(module
  (type $t (func (param i32) (result i32)))
  (import "env" "fail" (func $f (param i32) (result i32)))
  (table 1 funcref)
  (elem (i32.const 0) $f)
  (func (export "go") (param i32) (result i32) (return_call $f (local.get 0)))
  (func (export "go_ind") (param i32) (result i32)
    (return_call_indirect (type $t) (local.get 0) (i32.const 0)))
  (func $mid (param i32) (result i32) (local i32)
    (local.set 1 (i32.const 5))
    %s)
  (func (export "outer") (param i32) (result i32)
    (i32.add (call $mid (local.get 0)) (i32.const 100))))
"""
HOST_TAIL = assemble(HOST_TAIL_WAT % "(return_call $f (local.get 0))")
HOST_TWIN = assemble(HOST_TAIL_WAT % "(return (call $f (local.get 0)))")


def _host_tail_refs():
    rows = [[0], [3], [0], [0]]
    ref = {f: [O.Module(HOST_TAIL, tail_call=True).run(f, r) for r in rows] for f in ("go", "go_ind")}
    ref["outer"] = [O.Module(HOST_TWIN, tail_call=True).run("outer", r) for r in rows]
    assert [r[0] for r in ref["go"]] == [0, 0x8D, 0, 0] and ref["go"][0][1] == [7]
    assert ref["outer"][0][1] == [107]
    return rows, ref


def test_host_tail_calls_emulator(built):
    rows, ref = _host_tail_refs()
    from hostfuncs import emu_host
    for f in ("go", "go_ind", "outer"):
        got = emu_run(HOST_TAIL, f, rows, [I32], [I32], tail_call=True, host=emu_host(["fail"]))
        assert compare(ref[f], *got, [I32]) == [], f


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["compiled", "core", "step"])
def test_gpu_tail_calls_match_oracle(built, monkeypatch, engine):
    """Every tail-call shape on the GPU (direct, mutual with zeroed locals and stores,
    indirect through the table, from the entry function) against the oracle, on 192 lanes
    of mixed depths -- up to 100,000 frames deep, far past the device call stack's 4,096
    cells, which a tail call never uses. Engines: return_call compiled into the runs
    (default), the threaded core's handler (WB_JIT=0), the compiled C++ step (WB_JIT=0,
    WB_TC_TAIL=0)."""
    if engine != "compiled":
        monkeypatch.setenv("WB_JIT", "0")
    if engine == "step":
        monkeypatch.setenv("WB_TC_TAIL", "0")
    m = O.Module(TAIL, tail_call=True)
    rows = [[i % 3, (i * 977) % 1500] for i in range(190)] + [[0, 100000], [1, 100000]]
    ref = [m.run("run", r) for r in rows]
    assert compare(ref, *gpu_run(TAIL, "run", rows, [I32, I32], [I64], tail_call=True), [I64]) == []
    drows = [[n] for n in range(0, 640, 5)]
    ref = [m.run("direct", r) for r in drows]
    assert compare(ref, *gpu_run(TAIL, "direct", drows, [I32], [I64], tail_call=True), [I64]) == []


@pytest.mark.gpu
def test_gpu_tail_call_gate_and_host(built):
    from wasmedge_amd import batch
    with pytest.raises(batch.WasmEdgeError) as e:
        batch.BatchContext(TAIL, 64, device=0)
    assert e.value.code == 0x37
    import hostfuncs
    rows = [[0], [1], [3], [5], [2]]
    ref = [O.Module(INDIRECT_TRAPS, tail_call=True).run("go", r) for r in rows]
    ctx = batch.BatchContext(INDIRECT_TRAPS, 5, device=0, tail_call=True)
    try:
        hostfuncs.register(ctx)
        rets, st, cnt = ctx.execute("go", batch.make_values(rows, [I32]), 1)
        got = [[int(x) for x in r] for r in batch.ret_ints(rets)]
        assert compare(ref, got, st, cnt, ctx.memory_hash(), [I32], check_hash=False) == []
        assert [int(s) for s in st] == [0, 0x8C, 0x8A, 0x8B, 0x8D]
    finally:
        ctx.close()
    # host imports in tail position: entry frame = the reference, nested = the twin
    hrows, href = _host_tail_refs()
    for f in ("go", "go_ind", "outer"):
        ctx = batch.BatchContext(HOST_TAIL, len(hrows), device=0, tail_call=True)
        try:
            hostfuncs.register(ctx)
            rets, st, cnt = ctx.execute(f, batch.make_values(hrows, [I32]), 1)
            got = [[int(x) for x in r] if st[i] == 0 else [] for i, r in enumerate(batch.ret_ints(rets))]
            assert compare(href[f], got, st, cnt, ctx.memory_hash(), [I32], check_hash=False) == [], f
        finally:
            ctx.close()


# A direct call to a function defined AFTER its caller must zero the callee's locals too
# (helper.cpp:155-161 pushes ValueFromType zeros). Found while building tail calls: the
# lowering wrote the callee's local count into the CALL before lowering the callee (0),
# so such a callee saw the caller's stale cells in its locals.
FORWARD = assemble(r"""
(module
  (func (export "run") (param $x i32) (result i32) (local $a i32) (local $b i32) (local $c i32)
    (local.set $a (i32.const 11)) (local.set $b (i32.const 22)) (local.set $c (i32.const 33))
    (i32.add (call $later (local.get $x))
             (i32.add (local.get $a) (i32.add (local.get $b) (local.get $c)))))
  (func $later (param $p i32) (result i32) (local $acc i32) (local $k i32)
    (loop $l
      (local.set $acc (i32.add (local.get $acc) (local.get $p)))
      (local.set $k (i32.add (local.get $k) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $k) (i32.const 3))))
    (i32.add (local.get $acc) (i32.mul (local.get $k) (i32.const 1000)))))
""")


def test_forward_call_zeroes_locals_emulator(built):
    rows = [[x] for x in (0, 1, 7, 1000)]
    ref = [O.Module(FORWARD).run("run", r) for r in rows]
    assert [r[1][0] for r in ref] == [3 * x + 3000 + 66 for x in (0, 1, 7, 1000)]
    assert compare(ref, *emu_run(FORWARD, "run", rows, [I32], [I32]), [I32]) == []


@pytest.mark.gpu
@pytest.mark.parametrize("jit", ["1", "0"])
def test_gpu_forward_call_zeroes_locals(built, monkeypatch, jit):
    monkeypatch.setenv("WB_JIT", jit)
    rows = [[x] for x in range(130)]
    ref = [O.Module(FORWARD).run("run", r) for r in rows]
    assert compare(ref, *gpu_run(FORWARD, "run", rows, [I32], [I32]), [I32]) == []
