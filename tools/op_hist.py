"""Dynamic DBC op histogram of a workload on the host emulator (tuning aid, not a test).

usage: python tools/op_hist.py {blake3|qsort|collatz|mandel|fib} [n_instances]
Prints dispatches per DBC op (most frequent first) and wasm instrs per dispatch."""
import ctypes
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import helpers  # noqa: E402
from wasmedge_amd import workloads as W  # noqa: E402


def op_names():
    src = open(os.path.join(ROOT, "wasmedge_amd", "csrc", "dbc.h")).read()
    i = src.index("#define DBC_OPS(X)")
    return re.findall(r"X\((\w+)\)", src[i:src.index("enum DOp", i)])


CASES = {
    "blake3": lambda: (W.blake3_wasm(), "run", lambda i: [i, 20], [0x7F, 0x7F], [0x7F]),
    "qsort": lambda: (W.qsort_wasm(1), "sort", lambda i: [i, 4096], [0x7F, 0x7F], [0x7F]),
    "collatz": lambda: (W.collatz_wasm(), "collatz", lambda i: [i * 7 + 1, 10000], [0x7F, 0x7F], [0x7F]),
    "mandel": lambda: (W.mandel_wasm(), "tile", lambda i: [i * 977, 4096, 50], [0x7F, 0x7F, 0x7F], [0x7E]),
    "fib": lambda: (helpers_golden("fibonacci.wasm"), "fib", lambda i: [20], [0x7F], [0x7F]),
}


def helpers_golden(name):
    with open(os.path.join(ROOT, "tests", "golden", name), "rb") as f:
        return f.read()


def main():
    name = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    wasm, func, args, pt, rt = CASES[name]()
    E = helpers.emu_lib()
    nops = E.wb_emu_num_ops()
    h = np.zeros(nops, np.uint64)
    E.wb_emu_set_histogram(ctypes.c_void_p(h.ctypes.data))
    _, st, cnt, _ = helpers.emu_run(wasm, func, [args(i) for i in range(n)], pt, rt)
    E.wb_emu_set_histogram(None)
    names = op_names()
    tot = h.sum()
    print("instances %d  wasm instrs %d  dispatches %d  (%.2f instrs/dispatch)" %
          (n, int(cnt.sum()), int(tot), cnt.sum() / max(tot, 1)))
    for k in np.argsort(-h.astype(np.int64)):
        if h[k] == 0:
            break
        print("  %-20s %6.2f%%" % (names[k], 100.0 * h[k] / tot))


if __name__ == "__main__":
    main()
