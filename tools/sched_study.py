"""Compare wave scheduling policies on the BASELINE workloads: record each lane's DBC pc
trace on the host emulator (wb_emu_set_pc_trace), replay 64-lane waves through
tools/sched_sim.c, print lanes per dispatch and rounds. Tuning aid, not a test.

usage: python tools/sched_study.py [waves]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import helpers  # noqa: E402
from wasmedge_amd import workloads as W  # noqa: E402


class SimOut(ctypes.Structure):
    _fields_ = [("dispatches", ctypes.c_uint64), ("lane_dispatches", ctypes.c_uint64),
                ("rounds", ctypes.c_uint64)]


def cases(n):
    fib = open(os.path.join(ROOT, "tests", "golden", "fibonacci.wasm"), "rb").read()
    ids = range(n)
    return {
        "c1": (fib, "fib", [[12 + i % 11] for i in ids], [0x7F], [0x7F]),
        "c3": (W.qsort_wasm(), "sort", [[i, 1024] for i in ids], [0x7F, 0x7F], [0x7F]),
        "c4": (W.collatz_wasm(), "collatz", [[i, 10000] for i in ids], [0x7F, 0x7F], [0x7F]),
        "c5": (W.mandel_wasm(), "tile", [[(i * 2053 + 100000) % 262144, 4096, 50] for i in ids], [0x7F] * 3, [0x7E]),
    }


POLICIES = [("minpc", 0, 0, 0), ("loop,k1", 5, 1, 2), ("loop,k1,len<8", 8, 1, 2 + (8 << 8)),
            ("loop,k1,len<16", 8, 1, 2 + (16 << 8)), ("loop,k2,len<8", 8, 2, 2 + (8 << 8))]


def loops(wasm):
    """Innermost loop [head, end] around every pc, from the backward branches."""
    import re
    spans = []
    n = 0
    for ln in helpers.disasm(wasm).splitlines():
        m = re.match(r"\s*(\d+) (\w+).* imm=(\d+)", ln)
        if not m:
            continue
        pc, op, imm = int(m.group(1)), m.group(2), int(m.group(3))
        n = max(n, pc + 1)
        if (op == "JMP" or op.startswith("BR_")) and op != "BR_TABLE" and imm <= pc:
            spans.append((imm, pc))
    head, end, ph, pe = (np.full(n + 1, 0xFFFFFFFF, np.uint32) for _ in range(4))
    pe[:] = 0
    for x in range(n):
        inner = sorted((s for s in spans if s[0] <= x <= s[1]), key=lambda s: s[1] - s[0])
        if inner:
            head[x], end[x] = inner[0]
            outer = [s for s in inner if s[0] <= inner[0][0] and s[1] >= inner[0][1] and s != inner[0]]
            if outer:
                ph[x], pe[x] = outer[0]
    return head, end, ph, pe


def main():
    waves = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    only = sys.argv[2:] or None
    n = 64 * waves
    E = helpers.emu_lib()
    E.wb_emu_set_pc_trace.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    S = ctypes.CDLL(os.path.join(ROOT, "tools", "sched_sim.so"))
    S.sched_sim.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                            ctypes.POINTER(SimOut)]
    cap = 1 << 28
    buf = np.zeros(cap, np.uint32)
    for name, (wasm, fn, rows, pt, rt) in cases(n).items():
        if only and name not in only:
            continue
        lens = np.zeros(n, np.uint64)
        E.wb_emu_set_pc_trace(buf.ctypes.data, cap, lens.ctypes.data)
        helpers.emu_run(wasm, fn, rows, pt, rt)
        E.wb_emu_set_pc_trace(None, 0, None)
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum(lens)
        assert off[-1] < cap
        lh, le, ph, pe = loops(wasm)
        line = []
        for pname, pol, arg, arg2 in POLICIES:
            o = SimOut()
            S.sched_sim(buf.ctypes.data, off.ctypes.data, n, pol, arg, arg2, lh.ctypes.data, le.ctypes.data, ph.ctypes.data, pe.ctypes.data,
                        ctypes.byref(o))
            line.append("%s: lanes %.1f disp %.3g rounds %.3g" % (
                pname, o.lane_dispatches / o.dispatches, o.dispatches / waves, o.rounds / waves))
        print("%s (%d lanes, %.3g dispatches/lane)" % (name, n, off[-1] / n))
        for s in line:
            print("   ", s)
        sys.stdout.flush()


if __name__ == "__main__":
    main()
