"""Probe: throughput vs instances (waves per SIMD) and problem size, to tell latency-bound
from issue-bound workloads. Usage: python tools/probe_scale.py"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from wasmedge_amd import batch, workloads as W


def run(name, wasm, func, rows, types, **kw):
    n = len(rows)
    ctx = batch.BatchContext(wasm, n, **kw)
    ctx.set_args(func, batch.make_values(np.asarray(rows, dtype=np.int64), types))
    ctx.reset()
    tk = ctx.run()
    rets, st, cnt = ctx.results(1)
    tot = int(cnt.sum())
    print("%-12s n=%-7d instrs/inst=%.3e kernel=%.4fs -> %.3e instr/s traps=%d"
          % (name, n, tot / n, tk, tot / tk, int((st != 0).sum())), flush=True)
    ctx.close()


I32 = batch.I32
qs = W.qsort_wasm()
for n in (16384, 65536, 262144):
    run("qsort4k", qs, "sort", [[i, 4096] for i in range(n)], [I32, I32])
for n, el in ((1024, 65536), (1024, 262144), (4096, 262144)):
    run("qsort%dk" % (el // 1024), qs, "sort", [[i, el] for i in range(n)], [I32, I32])
fib = open(os.path.join(ROOT, "tests/golden/fibonacci.wasm"), "rb").read()
for n in (65536, 262144):
    run("fib-div", fib, "fib", [[20 + i % 11] for i in range(n)], [I32])
cz = W.collatz_wasm()
for n in (65536, 262144):
    run("collatz", cz, "collatz", [[i, 10000] for i in range(n)], [I32, I32])
mb = W.mandel_wasm()
for n in (65536, 262144):
    run("mandel", mb, "tile", [[i, 4096, 50] for i in range(n)], [I32, I32, I32])
