"""The MultiMemories proposal (include/common/enum.inc:555, off by default like TailCall,
configure.h:176-182): a module with three memories -- loads and stores of every width on
each, v128 forms, memory.size / memory.grow / memory.fill / memory.init per memory and
memory.copy within and across memories, an active data segment on memory 1, a trap on
memory 1's bound -- against the oracle's restatement (executor getMemInstByIdx,
memoryInstr.cpp, instantiate/data.cpp).

The reference reads a memarg's memory index AFTER the offset (instruction.cpp:144-156:
align, offset, then -- with the proposal and align >= 64 -- the index); the assembler
(wat.py) and both decoders follow it. Results fold samples of memories 1 and 2 into the
return value; the memory hash covers memory 0."""
import os

import numpy as np
import pytest

import oracle_py as O
from helpers import compare, emu_run
from wasmedge_amd.wat import assemble

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
I32 = 0x7F

MM_WAT = r"""
(module
  (memory $m0 1)
  (memory $m1 1 4)
  (memory $m2 2)
  (data (memory $m1) (i32.const 16) "hello multi")
  (data $p "passive-bytes!")
  (func (export "run") (param $seed i32) (param $n i32) (result i32)
    (local $k i32) (local $acc i32) (local $x i32)
    (local.set $x (i32.or (i32.mul (local.get $seed) (i32.const 2654435761)) (i32.const 1)))
    (block $done
      (loop $l
        (br_if $done (i32.ge_u (local.get $k) (local.get $n)))
        (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 13))))
        (local.set $x (i32.xor (local.get $x) (i32.shr_u (local.get $x) (i32.const 17))))
        (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 5))))
        (i32.store $m1 offset=64 (i32.shl (local.get $k) (i32.const 2)) (local.get $x))
        (i32.store8 $m2 (i32.and (local.get $x) (i32.const 0x1ffff)) (local.get $k))
        (i64.store $m0 offset=8 (i32.shl (i32.and (local.get $k) (i32.const 15)) (i32.const 3))
                   (i64.extend_i32_u (local.get $x)))
        (i32.store16 $m2 offset=3 (i32.and (local.get $k) (i32.const 0xfff)) (local.get $x))
        (local.set $acc (i32.add (local.get $acc)
          (i32.load16_u $m2 (i32.and (local.get $x) (i32.const 0x1fffe)))))
        (local.set $acc (i32.xor (local.get $acc)
          (i32.wrap_i64 (i64.load8_s $m1 offset=1 (i32.and (local.get $x) (i32.const 0xff))))))
        (local.set $k (i32.add (local.get $k) (i32.const 1)))
        (br $l)))
    (local.set $acc (i32.add (local.get $acc)
      (memory.grow $m1 (i32.and (local.get $seed) (i32.const 3)))))
    (local.set $acc (i32.add (local.get $acc)
      (memory.grow $m1 (i32.and (local.get $seed) (i32.const 1)))))
    (local.set $acc (i32.xor (local.get $acc) (i32.mul (memory.size $m1) (i32.const 1000))))
    (local.set $acc (i32.xor (local.get $acc) (i32.mul (memory.size $m2) (i32.const 7))))
    (memory.copy $m2 $m1 (i32.const 100) (i32.const 60) (local.get $n))
    (memory.copy $m0 $m2 (i32.const 200) (i32.const 90) (i32.const 64))
    (memory.copy $m1 $m1 (i32.const 70) (i32.const 64) (i32.const 40))
    (memory.copy $m1 $m0 (i32.const 3) (i32.const 200) (i32.const 17))
    (memory.fill $m2 (i32.const 300) (i32.const 0xAB) (i32.and (local.get $seed) (i32.const 63)))
    (memory.init $m2 $p (i32.const 500) (i32.const 2) (i32.const 9))
    (v128.store $m2 (i32.const 1024) (v128.load $m1 (i32.const 64)))
    (local.set $acc (i32.add (local.get $acc)
      (i32x4.extract_lane 1 (v128.load $m2 (i32.const 1024)))))
    (local.set $acc (i32.add (local.get $acc)
      (i32x4.extract_lane 2 (v128.load32_splat $m1 (i32.const 72)))))
    (local.set $acc (i32.add (local.get $acc) (i32.load $m1 (i32.const 16))))
    (local.set $acc (i32.add (local.get $acc) (i32.load $m2 (i32.const 500))))
    (local.set $acc (i32.add (local.get $acc) (i32.load $m0 (i32.const 200))))
    (local.set $acc (i32.add (local.get $acc) (i32.load $m1 (i32.const 3))))
    (i64.store $m0 (i32.const 400) (i64.load $m2 (i32.const 300)))
    ;; out of bounds on memory 1 for seed % 7 == 0 (its last 2 bytes hold no i32)
    (if (i32.eqz (i32.rem_u (local.get $seed) (i32.const 7)))
      (then (drop (i32.load $m1 (i32.sub (i32.shl (memory.size $m1) (i32.const 16))
                                         (i32.const 2))))))
    ;; ... and past memory 2's bound in a copy into it for seed % 11 == 0
    (if (i32.eqz (i32.rem_u (local.get $seed) (i32.const 11)))
      (then (memory.copy $m2 $m0 (i32.const 131070) (i32.const 0) (i32.const 4))))
    (local.get $acc))
)
"""


def mm_wasm():
    return assemble(MM_WAT)


def rows():
    return [[s, n] for s in range(96) for n in (0, 1, 5, 33, 200)]


def test_oracle_runs_the_module():
    """the restatement loads the module only with the proposal, and its lanes end both
    ways (results, and traps on memories 1 and 2)"""
    with pytest.raises(O.OracleError) as e:
        O.Module(mm_wasm())
    assert e.value.code == 0x51                      # multiple memories, proposal off
    m = O.Module(mm_wasm(), multi_memory=True)
    out = [m.run("run", r) for r in rows()]
    codes = {o[0] for o in out}
    assert codes == {0, 0x88}
    assert len({o[1][0] for o in out if o[0] == 0}) > 100


def test_oracle_memory_index_checks():
    """a memory index past the module's memories is InvalidMemoryIdx (0x47,
    formchecker.cpp:245-252), for an instruction and for an active data segment"""
    for bad in (MM_WAT.replace("(memory.size $m2)", "(memory.size 3)"),
                MM_WAT.replace("(memory.copy $m0 $m2", "(memory.copy 0 4"),
                MM_WAT.replace("(i32.load $m2 (i32.const 500))", "(i32.load 5 (i32.const 500))"),
                MM_WAT.replace('(data $p', '(data (memory 3) (i32.const 0) "x") (data $p')):
        with pytest.raises(O.OracleError) as e:
            O.Module(assemble(bad), multi_memory=True)
        assert e.value.code == 0x47
    more = MM_WAT.replace("(memory $m2 2)", "(memory $m2 2) (memory $m3 1)").replace(
        "(memory.size $m2)", "(memory.size 3)")
    assert O.Module(assemble(more), multi_memory=True).run("run", [1, 3])[0] == 0


def test_emulator_matches_the_oracle(built):
    """the lowering (XLD / XST / XLANE / XMEM_*) through the step code on the CPU emulator:
    bit-exact against the oracle (statuses, results, counts, memory-0 hashes)"""
    wasm = mm_wasm()
    rs = rows()
    ref = [O.Module(wasm, multi_memory=True).run("run", r) for r in rs]
    rets, st, cnt, h = emu_run(wasm, "run", rs, [I32, I32], [I32], multi_memory=True)
    assert compare(ref, rets, st, cnt, h, [I32], exact=True) == []
    with pytest.raises(RuntimeError) as e:   # proposal off: MultiMemories at load
        emu_run(wasm, "run", rs[:1], [I32, I32], [I32])
    assert "0x51" in str(e.value)


LANES_WAT = r"""
(module
  (memory $a 1)
  (memory $b 1)
  (func (export "run") (param $seed i32) (param $n i32) (result i32)
    (local $v v128)
    (i64.store $b (i32.const 32) (i64.extend_i32_u (i32.mul (local.get $seed) (i32.const 0x9e3779b1))))
    (i32.store $b (i32.const 40) (local.get $n))
    (local.set $v (v128.load8_lane $b 3 (i32.const 33) (v128.const i32x4 1 2 3 4)))
    (local.set $v (v128.load64_lane $b 1 (i32.const 36) (local.get $v)))
    (v128.store32_lane $b 2 (i32.and (local.get $n) (i32.const 0xfffe)) (local.get $v))
    (v128.store16_lane $a 5 (i32.const 8) (local.get $v))
    (i32.add (i32.load $b (i32.and (local.get $n) (i32.const 0xfffc)))
             (i32.add (i32.load $a (i32.const 8)) (i32x4.extract_lane 0 (local.get $v)))))
)
"""


def test_emulator_lane_forms():
    """v128.loadN_lane / storeN_lane on memories past the first (XLANE), and their bound"""
    wasm = assemble(LANES_WAT)
    rs = [[s, n] for s in range(40) for n in (0, 12, 65532, 65534)]
    ref = [O.Module(wasm, multi_memory=True).run("run", r) for r in rs]
    assert {r[0] for r in ref} == {0, 0x88}
    rets, st, cnt, h = emu_run(wasm, "run", rs, [I32, I32], [I32], multi_memory=True)
    assert compare(ref, rets, st, cnt, h, [I32], exact=True) == []


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["mm", "lanes"])
def test_gpu_multi_memory_exact(built, name):
    """on the GPU: memory 0 on every path, memories 1 and 2 in the per-lane step of the
    paged kernels; bit-exact against the oracle, and again after a Reset"""
    from wasmedge_amd import batch
    wasm = mm_wasm() if name == "mm" else assemble(LANES_WAT)
    rs = rows() if name == "mm" else [[s, n] for s in range(40) for n in (0, 12, 65532, 65534)]
    ref = [O.Module(wasm, multi_memory=True).run("run", r) for r in rs]
    ctx = batch.BatchContext(wasm, len(rs), multi_memory=True)
    try:
        for rep in range(2):
            if rep:
                ctx.reset()   # (Execute keeps instance state: the second run starts over)
            rets, st, cnt = ctx.execute("run", batch.make_values(rs, [I32, I32]), 1)
            h = ctx.memory_hash()
            ints = batch.ret_ints(rets)
            got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(rs))]
            assert compare(ref, got, st, cnt, h, [I32], exact=True) == [], rep
    finally:
        ctx.close()


def test_batch_refuses_without_the_proposal(built):
    """BatchCreate fails with MultiMemories (0x51) when the proposal is off (validator.cpp:
    107-113) -- before any device work"""
    from wasmedge_amd import batch
    with pytest.raises(batch.WasmEdgeError) as e:
        batch.BatchContext(mm_wasm(), 64)
    assert e.value.code == 0x51
