"""Loop-carried memory forwarding in the compiled runs (jit.cpp "Loop-carried memory
forwarding", DESIGN.md "Compiled runs").

A loop whose body calls an inlined leaf that reads and writes constant addresses gets a
second copy of its run in which the callee's loads are register moves (the words the
previous trip stored or loaded). These modules vary what the addresses do -- disjoint
words, a word one access stores and another loads (same address through different
cells), misaligned words (no forwarding: every trip leaves to the C++ step), words past
the one page of memory (every lane traps in the first trip) -- with per-lane trip counts
so that lanes leave the loop at different trips (the copies' split paths), and check
every lane against the oracle bit for bit with forwarding on and off."""
import ctypes
import os

import pytest

import oracle_py as O
from helpers import compare, gpu_run
from wasmedge_amd.wat import assemble

I32 = 0x7F
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS = [[(i * 2654435761 + 12345) & 0xFFFFFFFF] for i in range(160)]
CASES = [(64, 96), (64, 68), (64, 66), (65528, 96)]


def loop_module(a, b, div=False):
    # (div: the callee's result goes through 64-bit ops -- not plain 32-bit ones, so the
    # forwarding copy hands every aliased cell its own register before them)
    tail = ("(i32.wrap_i64 (i64.shr_u (i64.mul (i64.extend_i32_u (local.get $u)) "
            "(i64.const 0x9E3779B97F4A7C15)) (i64.const 17)))" if div else "(local.get $u)")
    return assemble(r"""
(module
  (memory 1)
  (func $leaf (param $a i32) (param $b i32) (param $x i32) (result i32)
    (local $t i32) (local $u i32)
    (local.set $t (i32.load offset=0 (local.get $a)))
    (local.set $u (i32.load offset=4 (local.get $b)))
    (i32.store offset=0 (local.get $b) (i32.add (local.get $t) (local.get $x)))
    (i32.store offset=8 (local.get $a) (i32.xor (i32.rotl (local.get $u) (i32.const 5)) (local.get $t)))
    (i32.add (i32.load offset=8 (local.get $a)) %s))
  (func (export "run") (param $s i32) (result i32)
    (local $i i32) (local $acc i32) (local $n i32) (local $pad i32)
    (i32.store (i32.const 64) (local.get $s))
    (i32.store (i32.const 100) (i32.mul (local.get $s) (i32.const 7)))
    (local.set $n (i32.add (i32.const 3) (i32.rem_u (local.get $s) (i32.const 29))))
    (loop $l
      (local.set $acc (i32.add (local.get $acc)
        (call $leaf (i32.const %d) (i32.const %d) (local.get $i))))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $i) (local.get $n))))
    (i32.add (local.get $acc) (i32.load (i32.const 96)))))
""" % (tail, a, b))


def random_loop_module(seed):
    """loop_module's shape with a random leaf: loads, stores and 32-bit ops over four
    locals, addresses a + k*4 / b + k*4 with constant a, b (coinciding words included)"""
    import random
    rnd = random.Random(seed)
    a, b = rnd.choice([(64, 96), (64, 72), (80, 64), (65520, 64)])
    ops = ["i32.add", "i32.sub", "i32.xor", "i32.or", "i32.and", "i32.mul", "i32.rotl", "i32.shl"]
    body = []
    for _ in range(rnd.randint(6, 14)):
        k = rnd.random()
        p, o = rnd.choice(["$a", "$b"]), 4 * rnd.randint(0, 3)
        t, u, v = ("$t%d" % rnd.randint(0, 3) for _ in range(3))
        if k < 0.35:
            body.append("(local.set %s (i32.load offset=%d (local.get %s)))" % (t, o, p))
        elif k < 0.6:
            body.append("(i32.store offset=%d (local.get %s) (%s (local.get %s) (local.get %s)))"
                        % (o, p, rnd.choice(ops), u, v))
        else:
            body.append("(local.set %s (%s (local.get %s) (local.get %s)))" % (t, rnd.choice(ops), u, v))
    return assemble(r"""
(module
  (memory 1)
  (func $leaf (param $a i32) (param $b i32) (param $x i32) (result i32)
    (local $t0 i32) (local $t1 i32) (local $t2 i32) (local $t3 i32)
    (local.set $t0 (local.get $x))
    %s
    (i32.xor (i32.xor (local.get $t0) (local.get $t1)) (i32.xor (local.get $t2) (local.get $t3))))
  (func (export "run") (param $s i32) (result i32)
    (local $i i32) (local $acc i32) (local $n i32) (local $pad i32)
    (i32.store (i32.const 64) (local.get $s))
    (i32.store (i32.const 76) (i32.mul (local.get $s) (i32.const 7)))
    (i32.store (i32.const 100) (i32.xor (local.get $s) (i32.const 0x5A5A)))
    (local.set $n (i32.add (i32.const 2) (i32.rem_u (local.get $s) (i32.const 17))))
    (loop $l
      (local.set $acc (i32.add (local.get $acc)
        (call $leaf (i32.const %d) (i32.const %d) (local.get $i))))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $i) (local.get $n))))
    (i32.add (local.get $acc) (i32.xor (i32.load (i32.const 64)) (i32.load (i32.const 100))))))
""" % ("\n    ".join(body), a, b))


def _copies(wasm):
    """forwarding copies of the compiled SIMT code (wb_jit_check's dump: labels Lb<k>c)"""
    L = ctypes.CDLL(os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch.so"))
    L.wb_jit_check.restype = ctypes.c_int
    L.wb_jit_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_uint32]
    path = "/tmp/wb_fwd_%d.s" % os.getpid()
    os.environ["WB_JIT_DUMP_SIMT"] = path
    try:
        err = ctypes.create_string_buffer(4096)
        assert L.wb_jit_check(wasm, len(wasm), 0, None, err, 4096) >= 0, err.value
        src = open(path).read()
        return sum(1 for ln in src.splitlines() if ln.strip().startswith('"Lb') and 'c:' in ln)
    finally:
        os.environ.pop("WB_JIT_DUMP_SIMT", None)


def test_forwarding_copies(built):
    """aligned disjoint or coinciding words forward; misaligned ones do not"""
    got = [_copies(loop_module(a, b)) for a, b in CASES]
    assert got[0] == 1 and got[1] == 1 and got[2] == 0, got
    assert _copies(loop_module(64, 68, True)) == 1


def test_random_loop_modules_forward(built):
    assert sum(_copies(random_loop_module(seed)) for seed in range(12)) >= 6


def test_loop_modules_trap_and_succeed():
    codes = set()
    for a, b in CASES:
        m = O.Module(loop_module(a, b))
        codes |= {m.run("run", r)[0] for r in ROWS[:8]}
    assert 0 in codes and 0x88 in codes


@pytest.mark.gpu
@pytest.mark.parametrize("knob", ["WB_FWD=1", "WB_FWD=0", "WB_SIMT=0", "WB_FWD_ALIAS=0"])
def test_gpu_forwarding_bit_exact(built, monkeypatch, knob):
    monkeypatch.setenv(*knob.split("="))
    for a, b, div in [(a, b, False) for a, b in CASES] + [(64, 68, True), (64, 96, True)]:
        wasm = loop_module(a, b, div)
        ref = [O.Module(wasm).run("run", r) for r in ROWS]
        rets, st, cnt, h = gpu_run(wasm, "run", ROWS, [I32], [I32])
        assert compare(ref, rets, st, cnt, h, [I32], exact=True) == [], (a, b)


@pytest.mark.gpu
def test_gpu_random_forwarding_bit_exact(built):
    for seed in range(12):
        wasm = random_loop_module(seed)
        ref = [O.Module(wasm).run("run", r) for r in ROWS]
        rets, st, cnt, h = gpu_run(wasm, "run", ROWS, [I32], [I32])
        assert compare(ref, rets, st, cnt, h, [I32], exact=True) == [], seed
