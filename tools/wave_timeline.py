"""When each batch wave ran (profiling build libwasmedge_batch_stats.so, -DWB_STATS: its
start / end s_memrealtime and HW_ID per wave). Prints, per workload, the kernel span, the
spread of wave durations, how many waves were resident over time (per SIMD: 1024 SIMDs)
and how the work is spread over the batch -- the evidence for where a divergent config's
time goes (tail vs. steady state). Usage: python tools/wave_timeline.py c1 c4 c5 [--out F]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["WB_BATCH_LIB"] = os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch_stats.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import bench  # noqa: E402
from wasmedge_amd import batch  # noqa: E402

ST_T0, ST_T1, ST_HW = 16, 17, 18
SIMDS = 1024


def timeline(name, n, elements=4096):
    a = argparse.Namespace(iters=1000, elements=elements, mt_n=100000)
    wasm, func, build, ptypes, desc, _ = bench.workload(name, a)
    L = batch.lib()
    L.wb_stats_read.restype = ctypes.c_uint32
    L.wb_stats_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    ctx = batch.BatchContext(wasm, n, device=0)
    ctx.set_args(func, batch.make_values(build(np.arange(n, dtype=np.int64)), ptypes))
    for _ in range(2):   # (the second run is measured: code objects and pages warm)
        ctx.reset()
        secs = ctx.run()
    _, st, cnt = ctx.results(1)
    nw = (n + 63) // 64
    raw = np.zeros(nw * 32 + 1024, np.uint64)
    L.wb_stats_read(ctx._h, raw.ctypes.data)
    ctx.close()
    w = raw[:nw * 32].reshape(nw, 32)
    t0, t1 = w[:, ST_T0].astype(np.float64), w[:, ST_T1].astype(np.float64)
    base = t0.min()
    t0, t1 = (t0 - base) / 100.0, (t1 - base) / 100.0   # microseconds (100 MHz)
    dur = t1 - t0
    span = t1.max()
    bins = 20
    res = []
    for k in range(bins):
        a0, a1 = span * k / bins, span * (k + 1) / bins
        ov = np.clip(np.minimum(t1, a1) - np.maximum(t0, a0), 0, None).sum() / (a1 - a0)
        res.append(round(ov / SIMDS, 3))
    q = np.percentile(dur, [0, 10, 50, 90, 99, 100])
    # work over the batch: mean wave duration per 1/16 of the wave ids
    strips = [round(float(s.mean()), 1) for s in np.array_split(dur, 16)]
    out = {"workload": name, "instances": n, "kernel_s": secs, "instr_per_s": float(cnt.sum()) / secs,
           "span_us": float(span), "wave_us_quantiles_0_10_50_90_99_100": [round(float(x), 1) for x in q],
           "mean_resident_waves_per_simd": round(float(dur.sum() / span / SIMDS), 3),
           "resident_per_simd_by_twentieth": res,
           "mean_wave_us_by_sixteenth_of_ids": strips,
           "waves_ending_in_last_10pct": int((t1 > 0.9 * span).sum()),
           "distinct_hw_ids": int(len(np.unique(w[:, ST_HW])))}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="+")
    ap.add_argument("--out")
    args = ap.parse_args()
    sizes = {"c1": 65536, "c2": 65536, "c3": 65536, "c4": 65536, "c5": 262144}
    res = [timeline(w, sizes.get(w, 65536)) for w in args.workloads]
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
