"""Dynamic fall-through pairs of DBC ops (op at pc, op at pc+1) weighted by how often the
pair executes back to back, over the BASELINE workloads on the host emulator. Tuning aid
for the threaded core's fused pair handlers (gen_tc.py PAIRS); not a test.

usage: python tools/pair_hist.py [top]"""
import ctypes
import os
import re
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import helpers  # noqa: E402
from wasmedge_amd import workloads as W  # noqa: E402

src = open(os.path.join(ROOT, "wasmedge_amd", "csrc", "dbc.h")).read()
i = src.index("#define DBC_OPS(X)")
NAMES = re.findall(r"X\((\w+)\)", src[i:src.index("enum DOp", i)])
CASES = {
    "c2": (W.blake3_wasm(), "run", [[k, 5] for k in range(4)], [0x7F, 0x7F], [0x7F]),
    "c3": (W.qsort_wasm(), "sort", [[k, 512] for k in range(4)], [0x7F, 0x7F], [0x7F]),
    "c4": (W.collatz_wasm(), "collatz", [[k * 7 + 1, 2000] for k in range(4)], [0x7F, 0x7F], [0x7F]),
    "c5": (W.mandel_wasm(), "tile", [[k * 977, 4096, 20] for k in range(2)], [0x7F] * 3, [0x7E]),
}


def main():
    top = int(sys.argv[1]) if len(sys.argv) > 1 else 25
    E = helpers.emu_lib()
    E.wb_emu_set_pc_histogram.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    for name, (wasm, fn, rows, pt, rt) in CASES.items():
        h = np.zeros(1 << 16, np.uint64)
        E.wb_emu_set_pc_histogram(h.ctypes.data, len(h))
        helpers.emu_run(wasm, fn, rows, pt, rt)
        E.wb_emu_set_pc_histogram(None, 0)
        ops = [int(m.group(1)) for m in re.finditer(r"^\s*\d+ (\w+)", helpers.disasm(wasm), re.M)
               if False]
        dis = helpers.disasm(wasm).splitlines()
        opn = {}
        for ln in dis:
            m = re.match(r"\s*(\d+) (\w+)", ln)
            if m:
                opn[int(m.group(1))] = m.group(2)
        tot = int(h.sum())
        pairs = Counter()
        for pc, x in opn.items():
            if pc + 1 in opn and h[pc] and h[pc + 1]:
                pairs[(x, opn[pc + 1], pc % 2)] += int(min(h[pc], h[pc + 1]))
        print("== %s: %d dispatches" % (name, tot))
        for (x, y, par), c in pairs.most_common(top):
            print("  %-20s %-20s even=%d %6.2f%%" % (x, y, par == 0, 100.0 * c / tot))


if __name__ == "__main__":
    main()
