"""Summarise a tools/prof_bench.sh output directory into profiles/.

usage: python tools/prof_summary.py <prof dir> <tag> [iters] [instances] [pages] [label]
(pages: linear-memory pages per instance, what wb_mem_hash_kernel reads; label: the
bench workload, default C2)
Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim),
profiles/<tag>_counters.md (per-kernel PMC means) and profiles/traffic_c2.json
(HBM bytes per interpreter launch, read by bench.py for roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE (KiB) come from
separate passes; gfx950 FETCH_SIZE reports half the bytes of coalesced reads, and we
calibrate that factor on our own access pattern with wb_mem_hash_kernel, which reads a
known byte count (every instance's pages, 4 B/lane lane-interleaved, the interpreter's
layout) -- so the correction is measured, not assumed.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    d, tag = sys.argv[1], sys.argv[2]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    inst = int(sys.argv[4]) if len(sys.argv) > 4 else 65536
    pages = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    label = sys.argv[6] if len(sys.argv) > 6 else None
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(d, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, tag + "_kernel_stats.csv"))
    C = {}
    for p in ["fetch", "write", "sq1", "sq2"]:
        C.update(counters(os.path.join(d, p, "run_counter_collection.csv")))
    stats0 = {r["Name"] for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv")))}
    # the interpreter kernel: the V-frame variant when the batch used it
    K = "wb_exec_vf_kernel" if "wb_exec_vf_kernel" in stats0 else "wb_exec_kernel"
    H = "wb_mem_hash_kernel"
    hash_bytes = 65536.0 * pages * inst      # every instance's pages (C2: 1 page each)
    fetch_factor = hash_bytes / (C[(H, "FETCH_SIZE")] * 1024.0)
    fetch = C[(K, "FETCH_SIZE")] * 1024.0 * fetch_factor
    write = C[(K, "WRITE_SIZE")] * 1024.0
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(d, "trace",
                                                                    "run_kernel_stats.csv")))}
    avg_ns = float(stats[K]["AverageNs"])
    waves = C[(K, "SQ_WAVES")]
    smem = C[(K, "SQ_INSTS_SMEM")]
    head = label or ("C2, %d instances x %d compressions" % (inst, iters))
    lines = ["# %s: rocprofv3 counters, `bench.py` (%s)" % (tag, head), "",
             "Per-kernel means over launches (counter passes run separately, see "
             "tools/prof_bench.sh).", "",
             "| kernel | counter | mean per launch |", "|---|---|---|"]
    for (k, c), v in sorted(C.items()):
        if k.startswith("wb_"):
            lines.append("| %s | %s | %.6g |" % (k, c, v))
    lines += ["", "## Derived (interpreter kernel `%s`)" % K, "",
              "* average duration (kernel trace): %.3f ms" % (avg_ns / 1e6),
              "* FETCH_SIZE calibration on wb_mem_hash_kernel: x%.4f (known %d B read)"
              % (fetch_factor, hash_bytes),
              "* HBM bytes per launch: fetch %.4g (corrected) + write %.4g = %.4g"
              % (fetch, write, fetch + write),
              "* waves %d; dispatches per wave ~ SQ_INSTS_SMEM/waves = %.0f" % (waves, smem / waves)]
    per = lambda c: C[(K, c)] / smem
    for c in ["SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_VALU", "SQ_INSTS_LDS",
              "SQ_INSTS_VMEM"]:
        lines.append("* %s per dispatch: %.2f" % (c, per(c)))
    wc = C[(K, "SQ_WAVE_CYCLES")]
    lines += ["* SQ_WAIT_ANY / SQ_WAVE_CYCLES = %.3f (parked on s_waitcnt)"
              % (C[(K, "SQ_WAIT_ANY")] / wc),
              "* SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES = %.3f" % (C[(K, "SQ_ACTIVE_INST_ANY")] / wc),
              "* SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES = %.3f" % (C[(K, "SQ_WAIT_INST_ANY")] / wc),
              "* shader cycles per dispatch (4 x wave quad-cycles / dispatches) = %.0f"
              % (4 * wc / smem)]
    open(os.path.join(prof, tag + "_counters.md"), "w").write("\n".join(lines) + "\n")
    json.dump({"iters": iters, "instances": inst, "hbm_bytes_per_launch": fetch + write,
               "fetch_bytes": fetch, "write_bytes": write, "fetch_factor": fetch_factor,
               "kernel_avg_ns": avg_ns, "source": tag,
               "valu_insts_per_launch": C[(K, "SQ_INSTS_VALU")],
               "salu_insts_per_launch": C[(K, "SQ_INSTS_SALU")],
               "wave_quad_cycles_per_launch": wc, "waves": waves},
              open(os.path.join(prof, "traffic_c2.json" if label is None else
                                "traffic_%s.json" % tag), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
