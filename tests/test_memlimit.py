"""The reference's page-limit test (test/memlimit/MemLimitTest.cpp:11-37) on the batched
path: WasmEdge_BatchConfigure.MaxMemoryPage plays RuntimeConfigure::MaxMemPage = 256.

* memory (1), limit 256:       grow(256) fails, grow(255) succeeds      (:23-26)
* memory (1 128), limit 256:   grow(128) fails, grow(127) succeeds      (:32-36)
* memory (257), limit 256:     no memory is allocated (:16-18) -> BatchCreate fails with
                               MemoryOutOfBounds (0x88); with no limit it instantiates (:20-21)

Per lane, grow(n) for varying n follows MemoryInstance::growPage
(include/runtime/instance/memory.h:88-113): -1 when min + n exceeds min(max, limit), else
the old size, and memory.size reports the new size."""
import pytest

from wasmedge_amd.wat import assemble

I32 = 0x7F
LIMIT = 256


def _module(limits):
    return assemble(r"""
(module
  (memory %s)
  (func (export "grow") (param i32) (result i32 i32)
    (memory.grow (local.get 0))
    (memory.size)))
""" % limits)


def _expect(mn, mx, n):
    cap = min(mx if mx is not None else 65536, LIMIT)
    return [0xFFFFFFFF, mn] if mn + n > cap else [mn, mn + n]


@pytest.mark.gpu
@pytest.mark.parametrize("mn,mx", [(1, None), (1, 128)])
def test_gpu_memlimit_grow(built, mn, mx):
    from wasmedge_amd import batch
    wasm = _module("%d %d" % (mn, mx) if mx else "%d" % mn)
    edge = mx if mx else LIMIT            # MemLimitTest's fail / succeed pair
    ns = [edge, edge - 1, 0, 1, 300, 65536, 0xFFFFFF00]   # no uint32 wrap of min + n
    rows = [[ns[i % len(ns)]] for i in range(200)]
    ctx = batch.BatchContext(wasm, len(rows), max_memory_page=LIMIT, device=0)
    try:
        rets, st, cnt = ctx.execute("grow", batch.make_values(rows, [I32]), 2)
        assert (st == 0).all()
        got = [[int(x) for x in r] for r in batch.ret_ints(rets)]
        assert got == [_expect(mn, mx, r[0]) for r in rows]
        assert _expect(mn, mx, edge)[0] == 0xFFFFFFFF and _expect(mn, mx, edge - 1)[0] == mn
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_memlimit_initial_over_limit(built):
    from wasmedge_amd import batch
    wasm = _module("257")
    with pytest.raises(batch.WasmEdgeError) as e:
        batch.BatchContext(wasm, 64, max_memory_page=LIMIT, device=0)
    assert e.value.code == 0x88
    ctx = batch.BatchContext(wasm, 64, device=0)      # no limit: allocated (:20-21)
    try:
        rets, st, cnt = ctx.execute("grow", batch.make_values([[0]] * 64, [I32]), 2)
        assert (st == 0).all()
        assert [[int(x) for x in r] for r in batch.ret_ints(rets)] == [[257, 257]] * 64
    finally:
        ctx.close()
