"""Debugging aid for trip mode (jit.cpp): run random test modules (tests/test_jit.py) on
the GPU under knob combinations and report, per seed, how many instances differ from the
oracle. usage: python tools/trip_debug.py <seed>..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys
sys.path[:0] = [%r, %r, %r]
import oracle_py as O, test_jit
from helpers import compare
from wasmedge_amd import batch
seed, n, g = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
rows = test_jit.ROWS[:n]
w = test_jit.random_module(seed)
ref = [O.Module(w).run("run", r) for r in rows]
ctx = batch.BatchContext(w, len(rows), memory_granule=g)
rets, st, cnt = ctx.execute("run", batch.make_values(rows, [0x7F]), 1)
h = ctx.memory_hash(); ints = batch.ret_ints(rets)
got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(rows))]
bad = compare(ref, got, st, cnt, h, [0x7E], exact=True)
lanes = sorted({b[0] for b in bad})
print("seed %%d n %%d g %%d runs %%d: %%d bad lanes %%s first %%s" %% (seed, n, g, ctx.compiled_runs(), len(lanes), lanes[:12], bad[:3]))
''' % (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"))

for seed in [int(a) for a in sys.argv[1:]]:
    for knobs in ({"WB_TRIP": "0"}, {"WB_TRIP": "1"}, {"WB_TRIP": "1", "WB_TRIP_SPLIT": "0"},
                  {"WB_TRIP": "1", "WB_JIT_SCHED": "0"},
                  {"WB_TRIP": "1", "WB_TRIP_SPLIT": "0", "WB_JIT_SCHED": "0"}):
        for n, g in ((256, 4), (64, 4), (1, 4), (256, 128)):
            env = dict(os.environ, **knobs)
            r = subprocess.run([sys.executable, "-c", CHILD, str(seed), str(n), str(g)], env=env,
                               capture_output=True, text=True, timeout=120)
            print(knobs, (r.stdout.strip() or r.stderr.strip()[-300:]), flush=True)
