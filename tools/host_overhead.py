"""Host-side cost of one bench step (Reset + Run) on a trivial module: the launch/sync
overhead that sits between interpreter kernels (tools/runs/gpu_r04_l.sh)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from wasmedge_amd import batch
from wasmedge_amd.wat import assemble

I32 = 0x7F
WAT = """(module (memory 1) (global $g (mut i32) (i32.const 0))
  (func (export "f") (param i32) (result i32)
    (global.set $g (i32.add (global.get $g) (local.get 0)))
    (i32.store (i32.const 16) (local.get 0))
    (global.get $g)))"""


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    ctx = batch.BatchContext(assemble(WAT), n, device=0)
    ctx.set_args("f", batch.make_values([[i] for i in range(n)], [I32]))
    for _ in range(20):
        ctx.reset(timed=False)
        ctx.run()
    for label, fn in (("run", lambda: ctx.run()),
                      ("reset+run", lambda: (ctx.reset(timed=False), ctx.run())),
                      ("reset(untimed)", lambda: ctx.reset(timed=False))):
        ts = []
        for _ in range(300):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        k = np.median([ctx.run() for _ in range(20)])
        print("kernel %.1f us;" % (1e6 * k), "%-16s n=%d median %.1f us  p10 %.1f us" % (label, n, 1e6 * np.median(ts), 1e6 * np.percentile(ts, 10)))
    ctx.close()


if __name__ == "__main__":
    main()
