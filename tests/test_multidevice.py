"""One batch over several devices from one process (SURVEY.md 8(b) NumDevices, 8(e)):
WasmEdge_BatchConfigure::Devices / DeviceCount / Partition (wasmedge_amd/csrc/multi.cpp).

The reference runs concurrent executes in one process (include/vm/vm.h:137-141 shared lock,
include/vm/async.h:25-40); here the instance ids are split over shards, one single-device
context each, by contiguous blocks of whole waves or by id mod G, with no collective --
outputs are gathered into the caller's [N] arrays in instance order. On the one-GPU test box
a device list [0, 0] puts two shards on one device: the results must be bit-identical to the
single-shard run and to the oracle, for both partitions."""
import os

import numpy as np
import pytest

import oracle_py as O
from helpers import compare
from wasmedge_amd import workloads as W
from wasmedge_amd.wat import assemble

I32, I64 = 0x7F, 0x7E


@pytest.mark.parametrize("G", [1, 2, 4, 8])
@pytest.mark.parametrize("part", [0, 1])
def test_placement_map(built, G, part):
    """Every id has one (shard, lane); a shard's lanes are 0..n_g-1; blocks are whole waves
    in id order, interleave is id mod G."""
    from wasmedge_amd import batch
    for n in (1, 63, 64, 65, 1000, 4096 + 17, 65536):
        seen = {}
        for i in range(n):
            g, l = batch.placement(n, G, part, i)
            assert 0 <= g < G and (g, l) not in seen
            seen[(g, l)] = i
            if part == 1:
                assert (g, l) == (i % G, i // G)
        sizes = [sum(1 for (gg, _) in seen if gg == g) for g in range(G)]
        for g in range(G):
            assert sorted(l for (gg, l) in seen if gg == g) == list(range(sizes[g]))
        if part == 0:
            span = -(-(-(-n // 64)) // G) * 64          # ceil(waves / G) whole waves
            assert all(seen[(g, l)] == g * span + l for (g, l) in seen)
        else:
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(batch.WasmEdgeError):
        batch.placement(10, 2, 0, 10)
    with pytest.raises(batch.WasmEdgeError):
        batch.placement(10, 0, 0, 1)


WHOAMI = assemble(r"""
(module
  (import "env" "whoami" (func $who (param i32) (result i32)))
  (import "env" "mem_sum" (func $sum (param i32 i32) (result i32)))
  (memory (export "memory") 1)
  (global $g (export "g") (mut i32) (i32.const 5))
  (func (export "go") (param $i i32) (result i32)
    (i32.store (i32.const 16) (i32.mul (local.get $i) (i32.const 3)))
    (global.set $g (i32.add (global.get $g) (local.get $i)))
    (i32.add (call $who (local.get $i)) (call $sum (i32.const 16) (i32.const 4)))))
""")


def _workloads():
    fib = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fibonacci.wasm"), "rb").read()
    return {
        "fib": (fib, "fib", [I32], [I32], lambda i: [i % 23]),
        "qsort": (W.qsort_wasm(), "sort", [I32, I32], [I32], lambda i: [i, (i * 37) % 700]),
        "collatz": (W.collatz_wasm(), "collatz", [I32, I32], [I32], lambda i: [i, 10000]),
        "mandel": (W.mandel_wasm(), "tile", [I32, I32, I32], [I64], lambda i: [i, 128, 50]),
    }


def _run(wasm, func, pt, rt, rows, **kw):
    from wasmedge_amd import batch
    ctx = batch.BatchContext(wasm, len(rows), **kw)
    try:
        rets, st, cnt = ctx.execute(func, batch.make_values(rows, pt), len(rt))
        return batch.ret_ints(rets).copy(), st.copy(), cnt.copy(), ctx.memory_hash().copy()
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("part", [0, 1])
def test_gpu_two_shards_one_device(built, part):
    """Devices [0, 0]: bit-identical to the single-shard run on every workload shape
    (recursion, per-lane memory, traps, f64x2), and to the oracle on a sample."""
    n = 200   # 4 waves: blocks give 128 + 72 lanes, interleave 100 + 100
    for name, (wasm, func, pt, rt, row) in _workloads().items():
        rows = [row(i) for i in range(n)]
        one = _run(wasm, func, pt, rt, rows, device=0)
        two = _run(wasm, func, pt, rt, rows, devices=[0, 0], partition=part)
        for a, b in zip(one, two):
            assert np.array_equal(a, b), name
        m = O.Module(wasm)
        sample = list(range(0, n, 13)) + [n - 1]
        ref = [m.run(func, rows[i]) for i in sample]
        got = [[int(x) for x in two[0][i]] if two[1][i] == 0 else [] for i in sample]
        assert compare(ref, got, two[1][sample], two[2][sample], two[3][sample], rt) == [], name


@pytest.mark.gpu
@pytest.mark.parametrize("part", [0, 1])
def test_gpu_two_shards_host_calls_and_state(built, part):
    """Host functions see batch-wide instance ids (WasmEdge_BatchMemoryGetInstance) and the
    calling instance's memory; per-instance memory, globals and pages route to the right
    shard; Reset and Interrupt reach every shard."""
    from wasmedge_amd import batch
    import hostfuncs
    n = 130
    ctx = batch.BatchContext(WHOAMI, n, devices=[0, 0], partition=part)
    try:
        ctx.add_host_function("env", "whoami", lambda mem, a: (0, [mem.instance * 1000]), 1, 1)
        ctx.add_host_function("env", "mem_sum", hostfuncs.mem_sum, 2, 1)
        rows = [[i] for i in range(n)]
        rets, st, cnt = ctx.execute("go", batch.make_values(rows, [I32]), 1)
        assert (st == 0).all()
        want = [i * 1000 + sum(((3 * i) & 0xFFFFFFFF).to_bytes(4, "little")) for i in range(n)]
        assert [int(x) for x in batch.ret_ints(rets)[:, 0]] == want
        for i in (0, 1, 64, 127, 129):
            assert ctx.memory(i, 16, 4) == (3 * i).to_bytes(4, "little")
            assert ctx.global_get("g", i)[0] == 5 + i
            assert ctx.memory_pages(i) == 1
        ctx.set_memory(77, 16, b"\x01\x00\x00\x00")
        ctx.global_set("g", None, 40, I32)
        rets, st, cnt = ctx.execute("go", batch.make_values(rows, [I32]), 1)
        assert [ctx.global_get("g", i)[0] for i in (0, 77, 129)] == [40, 117, 169]
        ctx.reset()
        assert [ctx.global_get("g", i)[0] for i in (0, 77, 129)] == [5, 5, 5]
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_shards_run_the_layout_trial(built):
    """mt19937 over two shards on one device through Reset cycles: the shards run the layout
    trial together (128-byte granules for the warm-up and the measured run, then 4-byte
    words; the first shard's verdict stands for both), every run bit-identical to the
    oracle sample."""
    import oracle_py as O
    from conftest import golden
    from helpers import compare, oracle_run
    from wasmedge_amd import batch
    wasm = golden("mt19937.wasm")
    n = 4096
    rows = [[0, 5489 + i, 3000] for i in range(n)]
    idx = list(range(0, n, 211)) + [n - 1]
    ref = oracle_run(O.Module(wasm), "mt19937", [rows[i] for i in idx])
    ctx = batch.BatchContext(wasm, n, devices=[0, 0], partition=batch.PARTITION_INTERLEAVE)
    try:
        vals = batch.make_values(rows, [0x7F, 0x7E, 0x7E])
        granules = []
        for k in range(4):
            if k:
                ctx.reset()
            rets, st, cnt = ctx.execute("mt19937", vals, 1)
            h = ctx.memory_hash()
            ints = batch.ret_ints(rets)
            got = [[int(ints[i][0])] if st[i] == 0 else [] for i in idx]
            assert compare(ref, got, st[idx], cnt[idx], h[idx], [0x7E]) == [], k
            granules.append(ctx.memory_granule())
        assert granules[:3] == [128, 128, 4] and granules[3] in (4, 128)
    finally:
        ctx.close()
