"""C1 anatomy: cycles per instruction on the critical lane of fib with every lane at one
n (uniform), with C1's n = 20 + id mod 11, and with only C1's n = 30 lanes working (the
others return at once). Kernel seconds x 2.4 GHz / the slowest lane's count. Tuning aid."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from wasmedge_amd import batch  # noqa: E402

fib = open(os.path.join(ROOT, "tests/golden/fibonacci.wasm"), "rb").read()
N = int(os.environ.get("N", 65536))
ids = np.arange(N)
cases = {"uni27": np.full(N, 27), "c1": 20 + ids % 11, "solo30": np.where(ids % 11 == 10, 30, 0),
         "pair2930": np.where(ids % 11 == 10, 30, np.where(ids % 11 == 9, 29, 0))}
for name, n in cases.items():
    ctx = batch.BatchContext(fib, N, device=0)
    ctx.set_args("fib", batch.make_values(n[:, None].astype(np.int64), [batch.I32]))
    best = 1e9
    for _ in range(2):
        ctx.reset()
        best = min(best, ctx.run())
    _, st, cnt = ctx.results(1)
    print("%-9s kernel %.4f s  instr/s %.3e  max count %.3e  cycles/instr on the slowest lane %.1f"
          % (name, best, cnt.sum() / best, cnt.max(), best * 2.4e9 / cnt.max()), flush=True)
    ctx.close()
