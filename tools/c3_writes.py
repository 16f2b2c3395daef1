"""Where C3's HBM writes come from (tuning aid, not a bench line): the quicksort module and
variants of it, each run once on 64K instances x --elements i32, one interpreter launch per
variant in this order (rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE of this script lists them in
the same order):
  base      the C3 module (workloads.qsort_wat)
  noswap    the partition's two swap stores dropped (the sort is wrong; its reads are not)
  nofill    the fill loop stores nothing (sorts zeroed memory: scans stop at once)
  trip0     base with trip mode off (WB_TRIP=0: SIMT scheduling only)
  scan0 / chain0 / split0   base without the trips' scan windows / forward chaining /
            stage A-B split (WB_TRIP_SCAN=0, WB_TRIP_CHAIN=0, WB_TRIP_SPLIT=0)
  hyb0      trips alone, no SIMT phases (WB_HYBRID=0)
usage: python tools/c3_writes.py [--elements N] [--only name,name]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def variants(n_el):
    from wasmedge_amd import workloads as W
    from wasmedge_amd.wat import assemble
    src = W.qsort_wat()
    swap = """            (local.set $t (i32.load (local.get $i)))
            (i32.store (local.get $i) (i32.load (local.get $j)))
            (i32.store (local.get $j) (local.get $t))"""
    assert swap in src
    noswap = src.replace(swap, """            (local.set $t (i32.load (local.get $i)))
            (drop (i32.load (local.get $j)))
            (drop (local.get $t))""")
    fill = "(i32.store (local.get $k) (local.get $x))"
    assert fill in src
    nofill = src.replace(fill, "(drop (local.get $x))")
    return [("base", assemble(src), {}), ("noswap", assemble(noswap), {}),
            ("nofill", assemble(nofill), {}), ("trip0", assemble(src), {"WB_TRIP": "0"}),
            ("scan0", assemble(src), {"WB_TRIP_SCAN": "0"}), ("chain0", assemble(src), {"WB_TRIP_CHAIN": "0"}),
            ("split0", assemble(src), {"WB_TRIP_SPLIT": "0"}), ("hyb0", assemble(src), {"WB_HYBRID": "0"})]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elements", type=int, default=4096)
    ap.add_argument("--instances", type=int, default=65536)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from wasmedge_amd import batch
    ids = np.arange(a.instances, dtype=np.int64)
    vals = batch.make_values(np.stack([ids, np.full_like(ids, a.elements)], 1), [batch.I32, batch.I32])
    for name, wasm, env in variants(a.elements):
        if a.only and name not in a.only.split(","):
            continue
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            ctx = batch.BatchContext(wasm, a.instances, max_memory_page=17, device=0)
            ctx.set_args("sort", vals)
            t = time.perf_counter()
            ks = ctx.run()
            wall = time.perf_counter() - t
            _, st, cnt = ctx.results(1)
            print("%-7s kernel %.4f s wall %.4f s instrs %.4g traps %d engine %s granule %d" % (
                name, ks, wall, float(cnt.sum()), int((st != 0).sum()), ctx.engine(),
                ctx.memory_granule()), flush=True)
            ctx.close()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v


if __name__ == "__main__":
    main()
