"""Debugging aid for trip mode: find the compiled run whose trip-mode code makes a random
test module (tests/test_jit.py) differ from the oracle, by leaving runs to the handlers
(WB_TRIP_EXCL) and bisecting. usage: python tools/trip_bisect.py <seed> [n lanes]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys
sys.path[:0] = [%r, %r, %r]
import oracle_py as O, test_jit
from helpers import compare
from wasmedge_amd import batch
seed, n = int(sys.argv[1]), int(sys.argv[2])
rows = test_jit.ROWS[:n]
w = test_jit.random_module(seed)
ref = [O.Module(w).run("run", r) for r in rows]
ctx = batch.BatchContext(w, len(rows))
rets, st, cnt = ctx.execute("run", batch.make_values(rows, [0x7F]), 1)
h = ctx.memory_hash(); ints = batch.ret_ints(rets)
got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(rows))]
bad = compare(ref, got, st, cnt, h, [0x7E], exact=True)
print("BAD" if bad else "GOOD", bad[:2])
''' % (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"))


def run(seed, n, excl, listfile=None):
    env = dict(os.environ, WB_TRIP="1", WB_TRIP_EXCL=",".join(map(str, excl)) or "999999")
    if listfile:
        env["WB_TRIP_LIST"] = listfile
    r = subprocess.run([sys.executable, "-c", CHILD, str(seed), str(n)], env=env,
                       capture_output=True, text=True, timeout=120)
    out = r.stdout.strip() or r.stderr.strip()[-300:]
    return out.startswith("BAD"), out


seed = int(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1
lf = tempfile.mktemp()
bad, out = run(seed, n, [], lf)
runs = [int(l.split()[0]) for l in open(lf)]
print("runs", runs, "all in:", out, flush=True)
if not bad:
    sys.exit(0)
# smallest set of runs that, kept in the trips, still fails: drop halves while it fails
keep = list(runs)
changed = True
while changed and len(keep) > 1:
    changed = False
    for half in (keep[: len(keep) // 2], keep[len(keep) // 2:]):
        b, o = run(seed, n, [p for p in runs if p not in half])
        print("keep", half, "->", o, flush=True)
        if b:
            keep, changed = half, True
            break
print("culprit runs kept in trip mode:", keep, flush=True)
for p in keep:
    b, o = run(seed, n, [q for q in runs if q != p])
    print("only", p, "->", o, flush=True)
