"""Model of SIMT group picks on C1's lanes (fib, n = base + id mod 11, one wave of 64): each
lane's sequence of compiled runs (the 5 runs of fibonacci.wasm's fib: entry test, leaf
return, first call, second call, add + return) with its call-stack height in slots (the
first call pushes 2, the second 3), replayed through a pick policy under the core's stop
rule (a group runs on until its next run ends at or above OTHER, the lowest waiting pc
above the group's pc, or it jumps to or below LOW, the lowest waiting pc; a split re-picks).
Prints group runs per run of the slowest lane (1.0 = the slowest lane never waits) and
picks per group run. LBF=1 models the pc-only split shortcut (the lower half goes on when
no lane waits at or below it). Tuning aid for jit.cpp sched_block, not a test.
usage: python tools/fib_sched_model.py [base]"""
import sys
sys.setrecursionlimit(10000)
PC = {0:0, 1:1, 2:3, 3:5, 4:8}; END = {0:0, 1:2, 2:4, 3:7, 4:10}
def trace(n):
    out = []
    def f(n, d):
        out.append((0, d))
        if n < 2:
            out.append((1, d)); return
        out.append((2, d)); f(n-2, d+2)
        out.append((3, d)); f(n-1, d+3)
        out.append((4, d))
    f(n, 0)
    return out
base = int(sys.argv[1]) if len(sys.argv) > 1 else 10
tr = {}
lanes = [base + i % 11 for i in range(64)]
T = [tr.setdefault(n, trace(n)) for n in lanes]
crit = max(len(t) for t in T)
INF = 1 << 30
import os
LBF = int(os.environ.get('LBF', '0'))
for pol in ["minpc", "mindepth", "maxdepth", "most"]:
    pos = [0]*64; steps = 0; picks = 0
    grp = None
    while True:
        live = [l for l in range(64) if pos[l] < len(T[l])]
        if not live: break
        if grp is None:
            groups = {}
            for l in live: groups.setdefault(T[l][pos[l]][0], []).append(l)
            if pol == "minpc": r = min(groups, key=lambda r: PC[r])
            elif pol == "mindepth": r = min(groups, key=lambda r: (min(T[l][pos[l]][1] for l in groups[r]), PC[r]))
            elif pol == "maxdepth": r = min(groups, key=lambda r: (-max(T[l][pos[l]][1] for l in groups[r]), PC[r]))
            else: r = min(groups, key=lambda r: (-len(groups[r]), PC[r]))
            grp = groups[r]; picks += 1
            wait = [PC[T[l][pos[l]][0]] for l in live if l not in grp]
            LOW = min(wait) if wait else INF
            up = [p for p in wait if p > PC[r]]
            OTHER = min(up) if up else INF
        # run the group's run
        steps += 1
        for l in grp: pos[l] += 1
        g2 = [l for l in grp if pos[l] < len(T[l])]
        if not g2: grp = None; continue
        nx = set(T[l][pos[l]][0] for l in g2)
        if len(nx) > 1:
            if LBF:
                lo, hi = sorted(nx, key=lambda r: PC[r])
                if LOW > PC[lo]:
                    grp = [l for l in g2 if T[l][pos[l]][0] == lo]
                    LOW = min(LOW, PC[hi]); OTHER = LOW
                    continue
            grp = None; continue
        t = nx.pop()
        if PC[t] <= LOW: OTHER = LOW
        if END[t] >= OTHER: grp = None; continue
        grp = g2
    print("%-9s steps/critical %.3f picks/step %.3f" % (pol, steps / crit, picks / steps))
