"""Entry-function layout (round-1 oracle bug). The reference runs the entry function until
its own `Func.getInstrs().end()` (lib/executor/engine/engine.cpp:40,45,1616): an iterator
into that function's private instruction vector, which no call can reach. The oracle keeps
every function in one flat code array, so it must not stop at `start + len` of the entry
function -- that is the first instruction of the NEXT function, and a call to it used to end
the loop with a bogus success. These modules put the callee right after the entry function
(and the entry right after its callee, the layout that always worked), at every depth the
reference's own frame rules touch: `call`, `return`, `call_indirect`, and a callee ending by
`br` to its function label."""
import pytest

import oracle_py as O
from helpers import compare, emu_run, gpu_run
from wasmedge_amd.wat import assemble

I32 = 0x7F

NEXT = assemble(r"""
(module
  (func $a (export "a") (result i32) (call $b) (i32.const 1) (i32.add))
  (func $b (result i32) (i32.const 7)))
""")

# every control path that leaves a callee, callee always directly after its caller
CHAIN = assemble(r"""
(module
  (type $t (func (param i32) (result i32)))
  (table 2 funcref)
  (elem (i32.const 0) $d $e)
  (func $entry (export "run") (param $x i32) (result i32)
    (i32.add (call $b (local.get $x)) (i32.const 100)))
  (func $b (param $x i32) (result i32)
    (if (result i32) (i32.and (local.get $x) (i32.const 1))
      (then (return (call $c (local.get $x))))
      (else (call_indirect (type $t) (local.get $x) (i32.and (i32.shr_u (local.get $x) (i32.const 1)) (i32.const 1))))))
  (func $c (param $x i32) (result i32)
    (block $out (result i32)
      (br $out (i32.mul (local.get $x) (i32.const 3)))))
  (func $d (param $x i32) (result i32) (br 0 (i32.sub (local.get $x) (i32.const 5))))
  (func $e (param $x i32) (result i32) (return (i32.xor (local.get $x) (i32.const 0xff)))))
""")

ROWS = [[x] for x in range(64)]


def test_oracle_call_to_next_function():
    """The VERDICT repro: a(){ b() + 1 } with b directly after a: 8 in 6 instructions
    (call, b's i32.const, b's end, i32.const, i32.add, a's end)."""
    code, vals, cnt, _ = O.Module(NEXT).run("a", [])
    assert (code, vals, cnt) == (0, [8], 6)


def test_oracle_chain_known_answers():
    m = O.Module(CHAIN)
    for x in range(16):
        code, vals, _, _ = m.run("run", [x])
        if x & 1:
            want = 3 * x
        elif (x >> 1) & 1:
            want = x ^ 0xFF
        else:
            want = (x - 5) & 0xFFFFFFFF
        assert code == 0 and vals == [(want + 100) & 0xFFFFFFFF], x


@pytest.mark.parametrize("wasm,func,rows", [(NEXT, "a", [[]] * 4), (CHAIN, "run", ROWS)],
                         ids=["next", "chain"])
def test_emulator_matches_oracle(built, wasm, func, rows):
    m = O.Module(wasm)
    ref = [m.run(func, r) for r in rows]
    got = emu_run(wasm, func, rows, [I32] * len(rows[0]), [I32])
    assert compare(ref, *got, [I32]) == []


@pytest.mark.gpu
@pytest.mark.parametrize("wasm,func,rows", [(NEXT, "a", [[]] * 64), (CHAIN, "run", ROWS)],
                         ids=["next", "chain"])
def test_gpu_matches_oracle(built, wasm, func, rows):
    m = O.Module(wasm)
    ref = [m.run(func, r) for r in rows]
    got = gpu_run(wasm, func, rows, [I32] * len(rows[0]), [I32], device=0)
    assert compare(ref, *got, [I32]) == []
