"""Debug probe for SIMT scan loops (jit.cpp): one random module of tests/test_jit.py on the
GPU against the oracle, mismatching lanes printed. Debug aid, not a test."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle_py as O
import test_jit as T
from wasmedge_amd import batch
seed = int(sys.argv[1]); gran = int(sys.argv[2]) if len(sys.argv) > 2 else 4
wasm = T.random_module(seed)
ref = [O.Module(wasm).run("run", r) for r in T.ROWS]
ctx = batch.BatchContext(wasm, len(T.ROWS), memory_granule=gran)
rets, st, cnt = ctx.execute("run", batch.make_values(T.ROWS, [T.I32]), 1)
ctx.close()
bad = 0
for i, (code, vals, rc, _) in enumerate(ref):
    if int(st[i]) != code or int(cnt[i]) != rc:
        bad += 1
        if bad <= 10:
            print("lane %d: status %d/%d count %d/%d diff %d" % (i, int(st[i]), code, int(cnt[i]), rc, int(cnt[i]) - rc))
print("bad", bad, "of", len(ref))
