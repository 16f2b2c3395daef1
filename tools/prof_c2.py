"""Profiling driver: one C2 launch (64K instances x ITERS compressions) after a warmup."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from wasmedge_amd import batch, workloads as W
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
ctx = batch.BatchContext(W.blake3_wasm(), n)
rows = np.zeros((n, 2), np.int64); rows[:, 0] = np.arange(n); rows[:, 1] = iters
ctx.set_args("run", batch.make_values(rows, [batch.I32, batch.I32]))
for _ in range(2):
    ctx.reset(); t = ctx.run()
_, st, cnt = ctx.results(1)
print("instrs", int(cnt.sum()), "kernel_s", t, "instr/s", cnt.sum() / t)
