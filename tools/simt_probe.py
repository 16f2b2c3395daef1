"""Debug probe for SIMT scheduling (KParams::simt): divergent fib on a few lanes with a
wall-clock limit, compared with the oracle. Tuning/debug aid, not a test."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np
import oracle_py
from wasmedge_amd import batch
wasm = open(os.path.join(ROOT, "tests", "golden", "fibonacci.wasm"), "rb").read()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
rows = [[6] for i in range(n)] if len(sys.argv) > 2 and sys.argv[2] == "uni" else [[3 + (i % 7)] for i in range(n)]
ctx = batch.BatchContext(wasm, n, device=0, time_limit=2.0)
print("runs", ctx.compiled_runs(), flush=True)
t = time.time()
rets, st, cnt = ctx.execute("fib", batch.make_values(rows, [batch.I32]), 1)
print("run %.3fs" % (time.time() - t), flush=True)
vals = batch.ret_ints(rets)
m = oracle_py.Module(wasm)
bad = 0
for i in range(n):
    code, ref, rcnt, _ = m.run("fib", rows[i])
    ok = int(st[i]) == code and int(vals[i][0]) == ref[0] and int(cnt[i]) == rcnt
    if not ok:
        bad += 1
        if bad <= 12:
            print("lane %d n=%d: status %d/%d value %d/%d count %d/%d" % (
                i, rows[i][0], int(st[i]), code, int(vals[i][0]), ref[0], int(cnt[i]), rcnt), flush=True)
print("bad lanes", bad, "of", n, flush=True)
