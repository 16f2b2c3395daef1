"""Debug aid: the memgrow module on 128 lanes with the virtual-memory layout, two pages
committed up front; prints per-lane page counts against the requested growth."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
from test_memgrow import grow_wasm, rows_for  # noqa: E402
from wasmedge_amd import batch  # noqa: E402
from wasmedge_amd.wat import assemble  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
simple = assemble("""(module (memory 1)
  (func (export "g") (param i32) (param i32) (result i32)
    (local $k i32) (local $r i32)
    (block $d (loop $l
      (br_if $d (i32.ge_u (local.get $k) (local.get 0)))
      (local.set $r (memory.grow (i32.const 7)))
      (br_if $d (i32.eq (local.get $r) (i32.const -1)))
      (local.set $k (i32.add (local.get $k) (i32.const 7)))
      (br $l)))
    (memory.size)))""")
for name, wasm, func in (("simple", simple, "g"), ("grow", grow_wasm(), "grow")):
    rows = rows_for(n, 1200, mult=419)
    ctx = batch.BatchContext(wasm, n, device=0, memory_reserve_pages=2)
    print(name, "engine", ctx.engine(), flush=True)
    rets, st, cnt = ctx.execute(func, batch.make_values(rows, [0x7F, 0x7F]), 1)
    ints = batch.ret_ints(rets)
    pages = [ctx.memory_pages(i) for i in range(n)]
    bad = [(i, rows[i][0], pages[i], int(ints[i][0]), int(st[i])) for i in range(n) if pages[i] < 1 + rows[i][0]]
    print(name, "lanes short of their pages:", len(bad), bad[:8], flush=True)
    print(name, "last error:", batch.lib().WasmEdge_BatchGetLastError(ctx._h), flush=True)
    ctx.close()
