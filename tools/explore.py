"""Exploratory throughput probe: each workload at a few sizes; kernel time (HIP events)
and aggregate instr/s. Usage: python tools/explore.py [names...]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from wasmedge_amd import batch, workloads as W

def run(name, wasm, func, rows, types, nret, reps=2, **kw):
    n = len(rows)
    ctx = batch.BatchContext(wasm, n, **kw)
    vals = batch.make_values(np.asarray(rows, dtype=np.int64), types)
    ctx.set_args(func, vals)
    best = None
    for r in range(reps):
        tr = ctx.reset()
        tk = ctx.run()
        best = tk if best is None else min(best, tk)
    rets, st, cnt = ctx.results(nret)
    tot = int(cnt.sum())
    print("%-10s n=%-7d instrs=%.3e kernel=%.4fs -> %.3e instr/s  (reset %.4fs, traps=%d, code=%d)"
          % (name, n, tot, best, tot / best, tr, int((st != 0).sum()), ctx.code_size()), flush=True)
    ctx.close()
    return tot / best

names = sys.argv[1:] or ["fib", "blake3", "collatz", "mandel", "qsort"]
I32, I64 = batch.I32, batch.I64
if "fib" in names:
    fib = open(os.path.join(ROOT, "tests/golden/fibonacci.wasm"), "rb").read()
    run("fib-uni", fib, "fib", [[25]] * 65536, [I32], 1)
    run("fib-div", fib, "fib", [[20 + i % 11] for i in range(65536)], [I32], 1)
if "blake3" in names:
    b3 = W.blake3_wasm()
    for n, it in [(65536, 100), (65536, 1000), (262144, 100)]:
        run("blake3", b3, "run", [[i, it] for i in range(n)], [I32, I32], 1)
if "collatz" in names:
    cz = W.collatz_wasm()
    run("collatz", cz, "collatz", [[i, 10000] for i in range(65536)], [I32, I32], 1)
if "mandel" in names:
    mb = W.mandel_wasm()
    run("mandel", mb, "tile", [[i, 2048, 50] for i in range(65536)], [I32, I32, I32], 1)
if "qsort" in names:
    qs = W.qsort_wasm()
    run("qsort4k", qs, "sort", [[i, 4096] for i in range(65536)], [I32, I32], 1)
