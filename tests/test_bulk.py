"""memory.fill / memory.copy (memoryInstr.cpp:59-101): the step code copies whole words
between byte-wise ends when source and destination share their alignment, in either
direction for overlapping ranges. Random ranges (aligned, misaligned, overlapping both
ways, empty, running off the end: 0x88) against the oracle on the emulator and the GPU,
memory hash exact."""
import random

import pytest

import oracle_py as O
from helpers import compare, emu_run, gpu_run
from wasmedge_amd.wat import assemble

I32 = 0x7F
BULK = assemble(r"""
(module
  (memory 1)
  (func (export "bulk") (param $d i32) (param $s i32) (param $n i32) (param $v i32) (param $mode i32)
        (result i32)
    (local $i i32)
    (loop $l   ;; a per-instance pattern over the first 4 KiB
      (i32.store8 (local.get $i) (i32.add (i32.mul (local.get $i) (i32.const 7)) (local.get $v)))
      (local.set $i (i32.add (local.get $i) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $i) (i32.const 4096))))
    (if (local.get $mode)
      (then (memory.copy (local.get $d) (local.get $s) (local.get $n)))
      (else (memory.fill (local.get $d) (local.get $v) (local.get $n))))
    (i32.xor (i32.load (i32.and (local.get $d) (i32.const 0xFFFC)))
             (i32.load (i32.const 2048)))))
""")


def _rows(seed=7, n=512):
    r = random.Random(seed)
    rows = []
    for i in range(n):
        d = r.randrange(0, 4096)
        k = r.random()
        if k < 0.4:
            s = (d & ~3) + r.choice([-64, -16, -4, 0, 4, 16, 64]) + (d & 3)   # same alignment, overlapping
        elif k < 0.7:
            s = r.randrange(0, 4096)
        else:
            s = d + r.choice([-3, -1, 1, 2, 5])
        s = max(0, s)
        n = r.choice([0, 1, 3, 4, 15, 16, 17, 63, 64, 65, 100, 256, 1000])
        if r.random() < 0.05:
            d = 65536 - r.randrange(0, 40)   # off the end for some n
        rows.append([d, s, n, r.randrange(256), i & 1])
    return rows


ROWS = _rows()


def _ref():
    m = O.Module(BULK)
    return [m.run("bulk", r) for r in ROWS]


def test_emulator_bulk_memory(built):
    ref = _ref()
    assert {r[0] for r in ref} == {0, 0x88}
    got = emu_run(BULK, "bulk", ROWS, [I32] * 5, [I32])
    assert compare(ref, *got, [I32], exact=True) == []


@pytest.mark.gpu
@pytest.mark.parametrize("granule", [4, 16, 128])
def test_gpu_bulk_memory(built, granule):
    ref = _ref()
    got = gpu_run(BULK, "bulk", ROWS, [I32] * 5, [I32], memory_granule=granule)
    assert compare(ref, *got, [I32], exact=True) == []
