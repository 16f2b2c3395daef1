"""Per-wave scheduler statistics of the interpreter on each config workload (profiling
build libwasmedge_batch_stats.so, -DWB_STATS). Prints, per workload: wasm instrs,
scheduler rounds, fast runs and mean active lanes, threaded-core entries, compiled-step
dispatches, slow steps, and the split of shader cycles (sched / fast run / slow step),
averaged over waves. Usage: python tools/sched_stats.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["WB_BATCH_LIB"] = os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch_stats.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from wasmedge_amd import batch, workloads as W  # noqa: E402

_src = open(os.path.join(ROOT, "wasmedge_amd", "csrc", "dbc.h")).read()
_i = _src.index("#define DBC_OPS(X)")
import re  # noqa: E402
OPS = re.findall(r"X\((\w+)\)", _src[_i:_src.index("enum DOp", _i)])
NAMES = ["rounds", "fast", "lanes", "tc", "cpp", "slow", "cyc_sched", "cyc_fast", "cyc_slow",
         "x_call", "x_ret", "x_post", "x_br", "x_other", "cyc_tc", "tc_sched"]
NST = 32   # per-wave stride of the stats buffer (batch_kernel.hip ST_N <= 32)


def run(name, wasm, func, rows, types):
    n = len(rows)
    L = batch.lib()
    L.wb_stats_read.restype = ctypes.c_uint32
    L.wb_stats_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    ctx = batch.BatchContext(wasm, n, device=0)
    ctx.set_args(func, batch.make_values(np.asarray(rows, dtype=np.int64), types))
    ctx.reset()
    t = ctx.run()
    _, st, cnt = ctx.results(1)
    nw = (n + 63) // 64
    raw = np.zeros(nw * NST + 1024, np.uint64)
    L.wb_stats_read(ctx._h, raw.ctypes.data)
    buf = raw[:nw * NST].reshape(nw, NST)
    hist = raw[nw * NST:]
    m = buf.astype(np.float64).mean(0)
    d = dict(zip(NAMES, m[:len(NAMES)]))
    cyc = (d["cyc_sched"] + d["cyc_fast"] + d["cyc_slow"]) * 16
    print("%-10s instr/s=%.3e wasm/inst=%.3e rounds=%.3e fast-lanes=%.1f tc=%.3e cpp=%.3e "
          "slow=%.3e | cycles/wave=%.3e sched=%.0f%% fast=%.0f%% slow=%.0f%% | cyc/round=%.0f"
          % (name, cnt.sum() / t, cnt.mean(), d["rounds"], d["lanes"] / max(d["fast"], 1),
             d["tc"], d["cpp"], d["slow"], cyc, 100 * 16 * d["cyc_sched"] / cyc,
             100 * 16 * d["cyc_fast"] / cyc, 100 * 16 * d["cyc_slow"] / cyc,
             cyc / max(d["rounds"], 1)), flush=True)
    print("           core exits at: call=%.3e ret=%.3e post_call=%.3e branch=%.3e other=%.3e"
          % (d["x_call"], d["x_ret"], d["x_post"], d["x_br"], d["x_other"]), flush=True)
    print("           inside the core %.0f%% of cycles; core returns for the scheduler %.3e per wave"
          % (100 * 16 * d["cyc_tc"] / cyc, d["tc_sched"]), flush=True)
    top = np.argsort(hist)[::-1][:8]
    print("           exit ops (per wave): " + " ".join(
        "%s=%.3g" % (OPS[k] if k < len(OPS) else k, hist[k] / nw) for k in top if hist[k]), flush=True)
    ctx.close()


I32 = batch.I32
N = 65536
fib = open(os.path.join(ROOT, "tests/golden/fibonacci.wasm"), "rb").read()
run("c2", W.blake3_wasm(), "run", [[i, 100] for i in range(N)], [I32, I32])
run("c1-div", fib, "fib", [[20 + i % 11] for i in range(N)], [I32])
run("fib-uni", fib, "fib", [[22] for i in range(N)], [I32])
run("c3-4k", W.qsort_wasm(), "sort", [[i, 4096] for i in range(N)], [I32, I32])
run("c4", W.collatz_wasm(), "collatz", [[i, 10000] for i in range(N)], [I32, I32])
run("c5", W.mandel_wasm(), "tile", [[i, 4096, 50] for i in range(N)], [I32, I32, I32])
run("c5-256k", W.mandel_wasm(), "tile", [[i, 4096, 50] for i in range(4 * N)], [I32, I32, I32])
