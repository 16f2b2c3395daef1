"""memory.grow at the reference's default configuration.

The reference grows a memory lazily up to its page limit: MemoryInstance::growPage
(include/runtime/instance/memory.h:87-115) fails past 65536 pages, past the module's max
and past RuntimeConfigure::MaxMemPage (default 65536, include/common/configure.h:123),
and otherwise commits the new pages of its 8 GiB+ mmap reservation on demand
(Allocator::resize, lib/system/allocator.cpp:101-129). The batched path reserves a
per-lane layout up front (WasmEdge_BatchConfigure::MemoryReservePages) and commits pages
past it from a device pool, 4 MiB rows per wave, through a page table (DESIGN.md "Linear
memory"). These tests run modules with no declared max under the default configuration,
lanes growing by 0..2,000 pages, bit-exact (returns, counts, memory hashes over every page)
against the oracle at its default page limit 65536 -- with the growth inside the reserved
layout, and forced through the pool.
"""
import os
import sys

import numpy as np
import pytest

from helpers import compare, emu_run
from wasmedge_amd.wat import assemble

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))

I32 = 0x7F

# grow(n, seed): n pages in chunks of 1 + seed % 97 (each grow's old size mixed in), then a
# word written in every page (at a seed-dependent offset and at its last word), read back;
# bulk ops and a misaligned i64 across the last page boundary; then a grow past 65536
# pages (-1) and memory.size.
GROW_WAT = r"""
(module
  (memory (export "memory") %s)
  (func (export "grow") (param $n i32) (param $seed i32) (result i32)
    (local $k i32) (local $chunk i32) (local $acc i32) (local $p i32) (local $pages i32)
    (local $step i32) (local $top i32)
    (local.set $chunk (i32.add (i32.rem_u (local.get $seed) (i32.const 97)) (i32.const 1)))
    (block $done
      (loop $g
        (br_if $done (i32.ge_u (local.get $k) (local.get $n)))
        (local.set $step (i32.sub (local.get $n) (local.get $k)))
        (if (i32.lt_u (local.get $chunk) (local.get $step)) (then (local.set $step (local.get $chunk))))
        (local.set $acc (i32.add (i32.mul (local.get $acc) (i32.const 31))
                                 (memory.grow (local.get $step))))
        (local.set $k (i32.add (local.get $k) (local.get $step)))
        (br $g)))
    (local.set $pages (memory.size))
    (local.set $top (i32.shl (local.get $pages) (i32.const 16)))
    (block $wd
      (loop $w
        (br_if $wd (i32.ge_u (local.get $p) (local.get $pages)))
        (i32.store
          (i32.add (i32.shl (local.get $p) (i32.const 16))
                   (i32.and (i32.add (i32.shl (local.get $seed) (i32.const 2))
                                     (i32.shl (local.get $p) (i32.const 3))) (i32.const 0xFFF8)))
          (i32.xor (local.get $p) (local.get $seed)))
        (i32.store offset=65532 (i32.shl (local.get $p) (i32.const 16))
          (i32.mul (local.get $p) (i32.const 3)))
        (local.set $p (i32.add (local.get $p) (i32.const 1)))
        (br $w)))
    ;; bulk memory across the last pages (the reserved layout / pool boundary for most lanes)
    (if (i32.ge_u (local.get $pages) (i32.const 3))
      (then
        (memory.fill (i32.sub (local.get $top) (i32.const 70001))
                     (local.get $seed) (i32.const 70000))
        (memory.copy (i32.const 1000) (i32.sub (local.get $top) (i32.const 65601)) (i32.const 300))
        (memory.copy (i32.sub (local.get $top) (i32.const 131075)) (i32.const 996) (i32.const 200))
        (local.set $acc (i32.add (local.get $acc)
          (i32.wrap_i64 (i64.load (i32.sub (local.get $top) (i32.const 65539))))))))
    (local.set $p (i32.const 0))
    (block $rd
      (loop $r
        (br_if $rd (i32.ge_u (local.get $p) (local.get $pages)))
        (local.set $acc (i32.add (i32.mul (local.get $acc) (i32.const 17))
          (i32.add
            (i32.load (i32.add (i32.shl (local.get $p) (i32.const 16))
                               (i32.and (i32.add (i32.shl (local.get $seed) (i32.const 2))
                                                 (i32.shl (local.get $p) (i32.const 3))) (i32.const 0xFFF8))))
            (i32.load offset=65532 (i32.shl (local.get $p) (i32.const 16))))))
        (local.set $p (i32.add (local.get $p) (i32.const 1)))
        (br $r)))
    (i32.add (i32.add (local.get $acc) (memory.grow (i32.const 65536))) (memory.size)))
  (func (export "peek") (param $a i32) (result i32) (i32.load (local.get $a))))
"""


def grow_wasm(limits="1"):
    return assemble(GROW_WAT % limits)


def rows_for(n_lanes, max_pages, mult=613):
    return [[(i * mult) % (max_pages + 1), 0x5EED + 7 * i] for i in range(n_lanes)]


def oracle_rows(wasm, rows, threads=8):
    import oracle_py
    m = oracle_py.Module(wasm)
    params = np.zeros((len(rows), 2, 2), np.uint64)
    for i, r in enumerate(rows):
        params[i, 0, 0], params[i, 1, 0] = r
    out = m.run_batch("grow", params, len(rows), threads=threads)
    return [(int(out["codes"][i]), [int(out["results"][i, 0, 0])], int(out["counts"][i]),
             int(out["hashes"][i])) for i in range(len(rows))]


def test_emu_default_limit_grows_like_the_oracle(built):
    """The step code's memory.grow (the emulator) at the default page limit: a module with
    no max grows far past its initial size, as the reference does."""
    wasm = grow_wasm()
    rows = rows_for(12, 300)
    ref = oracle_rows(wasm, rows, threads=4)
    rets, st, cnt, h = emu_run(wasm, "grow", rows, [I32, I32], [I32])
    assert compare(ref, rets, st, cnt, h, [I32]) == []
    assert max(r[0] for r in rows) > 100


def _gpu_grow(wasm, rows, ref, **kw):
    from wasmedge_amd import batch
    ctx = batch.BatchContext(wasm, len(rows), device=0, **kw)
    try:
        vals = batch.make_values(rows, [I32, I32])
        for rep in range(2):   # a Reset returns every page; the second run must match again
            rets, st, cnt = ctx.execute("grow", vals, 1)
            h = ctx.memory_hash()
            ints = batch.ret_ints(rets)
            got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(rows))]
            assert compare(ref, got, st, cnt, h, [I32]) == [], rep
            pages = [ctx.memory_pages(i) for i in range(len(rows))]
            assert pages == [1 + r[0] for r in rows]
            # the host's view of the grown pages (WasmEdge_BatchGetMemory): the last two
            # pages as the oracle's memory holds them
            import oracle_py
            m = oracle_py.Module(wasm)
            for i in (0, len(rows) // 2, len(rows) - 1):
                _, _, _, mem = m.run_with_memory("grow", rows[i])
                lo = max(0, len(mem) - 131072)
                assert ctx.memory(i, lo, len(mem) - lo) == mem[lo:], i
            ctx.reset()
        # host writes into a grown page, the module reads them back
        rets, st, cnt = ctx.execute("grow", vals, 1)
        i = max(range(len(rows)), key=lambda k: rows[k][0])
        addr = (rows[i][0] << 16) + 12
        ctx.set_memory(i, addr, b"\x78\x56\x34\x12")
        rets, st, cnt = ctx.execute("peek", batch.make_values([[addr]] * len(rows), [I32]), 1)
        assert int(batch.ret_ints(rets)[i][0]) == 0x12345678
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_grow_default_config(built):
    """No max, default configuration (MaxMemoryPage 0 = 65536): lanes grow by 0..2,000
    pages inside the reserved layout; bit-exact against the oracle's default limit."""
    wasm = grow_wasm()
    rows = rows_for(64, 2000)
    _gpu_grow(wasm, rows, oracle_rows(wasm, rows))


@pytest.mark.gpu
@pytest.mark.parametrize("relayout", ["1", "0"])
def test_gpu_grow_through_the_pool(built, monkeypatch, relayout):
    """The same with two reserved pages: lanes park at memory.grow and the host gives them
    the pages -- by growing the reserved layout (relayout 1: the old rows copied over, every
    engine then addresses the grown pages directly) or from the device pool (WB_RELAYOUT=0:
    rows through the page table, which widens) -- over two waves; bit-exact against the
    oracle, and again after a Reset."""
    monkeypatch.setenv("WB_RELAYOUT", relayout)
    wasm = grow_wasm()
    rows = rows_for(128, 1200, mult=419)
    _gpu_grow(wasm, rows, oracle_rows(wasm, rows), memory_reserve_pages=2)


@pytest.mark.gpu
def test_gpu_layout_takes_the_grown_pages(built):
    """Lanes that grow past the reserved layout (two pages): the service round grows the
    layout to every page they ask for (WasmEdge_BatchGetReservedPages), where every engine
    addresses it directly; bit-exact on every run, across Resets. With the growth done in
    the run, a Reset after a pool-served run (WB_RELAYOUT=0 for the first run) re-lays memory
    with the pages the lanes reached."""
    from wasmedge_amd import batch
    wasm = grow_wasm()
    rows = rows_for(128, 300, mult=419)
    ref = oracle_rows(wasm, rows)
    top = 1 + max(r[0] for r in rows)
    ctx = batch.BatchContext(wasm, len(rows), device=0, memory_reserve_pages=2)
    try:
        vals = batch.make_values(rows, [I32, I32])
        assert ctx.reserved_pages() == 2
        for rep in range(3):
            rets, st, cnt = ctx.execute("grow", vals, 1)
            ints = batch.ret_ints(rets)
            got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(rows))]
            assert compare(ref, got, st, cnt, ctx.memory_hash(), [I32]) == [], rep
            assert ctx.reserved_pages() >= top, rep
            ctx.reset()
    finally:
        ctx.close()
    os.environ["WB_RELAYOUT"] = "0"
    try:
        ctx = batch.BatchContext(wasm, len(rows), device=0, memory_reserve_pages=2)
        vals = batch.make_values(rows, [I32, I32])
        rets, st, cnt = ctx.execute("grow", vals, 1)
        assert ctx.reserved_pages() == 2
    finally:
        del os.environ["WB_RELAYOUT"]
    try:
        ctx.reset()   # (the pool-served run's pages: the Reset takes them into the layout)
        assert ctx.reserved_pages() == top
        rets, st, cnt = ctx.execute("grow", vals, 1)
        ints = batch.ret_ints(rets)
        got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(rows))]
        assert compare(ref, got, st, cnt, ctx.memory_hash(), [I32]) == []
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_grow_pool_exhausted(built):
    """A cap on the pool (MemoryPoolBytes = 16 rows of 4 MiB): growPage's allocation
    failure (memory.h:104-109) -- lanes asking for more pages than the wave can get see
    -1, the others grow."""
    from wasmedge_amd import batch
    wasm = assemble("""(module (memory 1)
      (func (export "g") (param i32) (result i32 i32)
        (memory.grow (local.get 0)) (memory.size)))""")
    ctx = batch.BatchContext(wasm, 64, device=0, memory_reserve_pages=1, memory_pool_bytes=16 << 22)
    try:
        rets, st, cnt = ctx.execute("g", batch.make_values([[i] for i in range(64)], [I32]), 2)
        assert (st == 0).all()
        got = [[int(x) for x in r] for r in batch.ret_ints(rets)]
        assert got == [[1, 1 + i] if i <= 16 else [0xFFFFFFFF, 1] for i in range(64)]
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_max_65536_module_at_64k_instances(built):
    """A module declaring max 65536 instantiates at 64K instances (nothing like 4 GiB
    per lane is reserved up front); lanes grow by 0..6 pages, some waves past the reserved
    layout into the pool; a sample is bit-exact against the oracle."""
    from wasmedge_amd import batch
    wasm = grow_wasm("1 65536")
    n = 65536
    rows = [[i % 7, i] for i in range(n)]
    sample = list(range(0, n, 4099)) + [n - 1]
    ref = oracle_rows(wasm, [rows[i] for i in sample])
    ctx = batch.BatchContext(wasm, n, device=0)
    try:
        rets, st, cnt = ctx.execute("grow", batch.make_values(rows, [I32, I32]), 1)
        h = ctx.memory_hash()
        ints = batch.ret_ints(rets)
        got = [[int(ints[i][0])] for i in sample]
        assert compare(ref, got, st[sample], cnt[sample], h[sample], [I32]) == []
        assert (st == 0).all()
    finally:
        ctx.close()
