"""Summarise a tools/prof_bench.sh output directory into profiles/.

usage: python tools/prof_summary.py <prof dir> <tag> <pages>
  pages: linear-memory pages per instance at the end of the run (what wb_mem_hash_kernel
  reads; 0 for a module without memory)

Reads the bench line the trace pass printed (its configuration identifies the profile)
and writes:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats of the trace pass, verbatim
  profiles/<tag>_counters.md        per-kernel PMC means + the derived figures
  profiles/prof_<workload>.json     what bench.py reads for that configuration: HBM bytes,
                                    VALU instructions, active lanes per VALU instruction,
                                    occupancy, VMEM latency, wait fraction per launch

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE (KiB) come from
separate passes; gfx950 FETCH_SIZE reports half the bytes of coalesced reads, so the fetch
figure is FETCH_SIZE x 2 as the guide prescribes. wb_mem_hash_kernel, which streams a
known byte count (every instance's pages, 16 B per lane, nontemporal), is the check: its
known bytes / FETCH_SIZE is reported next to the x2 (`fetch_check`).

Exec-mask efficiency: SQ_THREAD_CYCLES_VALU counts, per VALU instruction, its cycles
times its active lanes; divided by SQ_ACTIVE_INST_VALU (cycles of VALU instructions) it
is the mean number of active lanes per VALU instruction (64 = no divergence; the
rocprofv3 derived metric VALUUtilization is this over 64).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
XCDS = 8
SIMDS = 256 * 4


# PROF_LAST=n: the interpreter kernel's figures over its last n launches only (the bench's
# timed steps: a run before them may have had another memory layout, the layout trial)
LAST = int(os.environ.get("PROF_LAST", "0"))
EXEC = ("wb_exec_vf_kernel", "wb_exec_kernel", "wb_exec_hbm_kernel", "wb_exec_vf_pg_kernel",
        "wb_exec_pg_kernel", "wb_exec_hbm_pg_kernel")


def counters(path):
    agg = collections.defaultdict(list)
    if not os.path.exists(path):
        return {}
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    for r in rows:
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v[-LAST:] if LAST and k[0] in EXEC else v) / len(v[-LAST:] if LAST and k[0] in EXEC else v)
            for k, v in agg.items()}


def last_avg_ns(d, kernel):
    """Mean duration of the kernel's last LAST launches in the trace pass."""
    rows = [r for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv")))
            if r["Kernel_Name"] == kernel]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ds = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[-LAST:]]
    return sum(ds) / len(ds)


def bench_line(path):
    for line in open(path):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit("no bench line in " + path)


def profile_key(cfg):
    """The configuration fields a profile is valid for (bench.py compares them)."""
    return {k: cfg[k] for k in ("workload", "instances_per_gpu", "elements", "iters", "draws") if k in cfg}


def main():
    d, tag, pages = sys.argv[1], sys.argv[2], int(sys.argv[3])
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    line = bench_line(os.path.join(d, "trace.log"))
    cfg = line["config"]
    inst = cfg["instances_per_gpu"]
    wl = line.get("workload_key") or cfg["workload"].split()[0].lower()
    shutil.copy(os.path.join(d, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, tag + "_kernel_stats.csv"))
    C = {}
    for p in ["fetch", "write", "sq1", "sq2", "util", "lat"]:
        C.update(counters(os.path.join(d, p, "run_counter_collection.csv")))
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(d, "trace",
                                                                    "run_kernel_stats.csv")))}
    K = next(k for k in EXEC if k in stats)
    H = "wb_mem_hash_kernel"
    g = lambda c, k=K: C.get((k, c))
    hash_bytes = 65536.0 * pages * inst
    fetch_factor = 2.0
    fetch_check = hash_bytes / (g("FETCH_SIZE", H) * 1024.0) if pages and g("FETCH_SIZE", H) else None
    fetch = g("FETCH_SIZE") * 1024.0 * fetch_factor
    write = g("WRITE_SIZE") * 1024.0
    avg_ns = last_avg_ns(d, K) if LAST else float(stats[K]["AverageNs"])
    waves = g("SQ_WAVES")
    wc = g("SQ_WAVE_CYCLES")                 # quad-cycles, summed over waves
    gui = g("GRBM_GUI_ACTIVE")               # cycles, summed over the XCDs
    valu = g("SQ_INSTS_VALU")
    out = {"config": profile_key(cfg), "source": tag, "kernel": K, "kernel_avg_ns": avg_ns,
           "launches_averaged": ("the last %d" % LAST) if LAST else "all",
           "waves": waves, "hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch,
           "write_bytes": write, "fetch_factor": fetch_factor, "fetch_check": fetch_check,
           "valu_insts_per_launch": valu, "salu_insts_per_launch": g("SQ_INSTS_SALU"),
           "vmem_insts_per_launch": g("SQ_INSTS_VMEM"), "lds_insts_per_launch": g("SQ_INSTS_LDS"),
           "branch_insts_per_launch": g("SQ_INSTS_BRANCH"),
           "wave_quad_cycles_per_launch": wc,
           "wait_any_frac": g("SQ_WAIT_ANY") / wc, "active_any_frac": g("SQ_ACTIVE_INST_ANY") / wc,
           "active_valu_frac": g("SQ_ACTIVE_INST_VALU") / wc,
           "bench_ms_per_step": line["ms_per_step"],
           # the HIP-event kernel time the traced run's own bench line measured (same
           # process, same launches as the trace): the two clocks side by side
           "bench_kernel_ms": line.get("kernel_ms")}
    # mean resident waves per SIMD over the kernel: wave cycles / (kernel cycles x SIMDs)
    if gui:
        out["waves_per_simd"] = 4.0 * wc / (gui / XCDS) / SIMDS
    tc = g("SQ_THREAD_CYCLES_VALU")
    if tc is not None and g("SQ_ACTIVE_INST_VALU"):
        out["lanes_per_valu"] = tc / g("SQ_ACTIVE_INST_VALU")
        out["valu_utilization"] = out["lanes_per_valu"] / 64.0
    if g("TCC_HIT_sum") is not None:
        h, m = g("TCC_HIT_sum"), g("TCC_MISS_sum")
        out["l2_hit_rate"] = h / max(h + m, 1.0)
    if g("VmemLatency") is not None:
        out["vmem_latency_cycles"] = g("VmemLatency")
    lines = ["# %s: rocprofv3 counters, `bench.py` %s" % (tag, json.dumps(out["config"])), "",
             "Per-kernel means over launches (counter passes run separately, see "
             "tools/prof_bench.sh)%s." % (
                 "; the interpreter kernel over its last %d launches (the timed steps)" % LAST
                 if LAST else ""), "",
             "| kernel | counter | mean per launch |", "|---|---|---|"]
    for (k, c), v in sorted(C.items()):
        if k.startswith("wb_"):
            lines.append("| %s | %s | %.6g |" % (k, c, v))
    lines += ["", "## Derived (interpreter kernel `%s`)" % K, "",
              "* average duration (kernel trace): %.3f ms; the same run's HIP-event kernel time "
              "%s ms; bench ms per step in the trace pass %.3f" % (
                  avg_ns / 1e6, "%.3f" % line["kernel_ms"] if line.get("kernel_ms") else "n/a",
                  line["ms_per_step"]),
              "* FETCH_SIZE correction: x%.1f (the guide); check: wb_mem_hash_kernel streams a "
              "known %d B = FETCH_SIZE x %s" % (fetch_factor, hash_bytes,
                                                "%.4f" % fetch_check if fetch_check else "n/a"),
              "* HBM bytes per launch: fetch %.4g (corrected) + write %.4g = %.4g"
              % (fetch, write, fetch + write),
              "* waves %d; resident waves per SIMD %.2f" % (waves, out.get("waves_per_simd", 0)),
              "* VALU instructions per launch %.4g; issue rate %.4g lane-op/s (x64 / duration)"
              % (valu, valu * 64 / (avg_ns * 1e-9))]
    for k in ("lanes_per_valu", "l2_hit_rate", "vmem_latency_cycles", "wait_any_frac",
              "active_any_frac", "active_valu_frac"):
        if k in out:
            lines.append("* %s = %.4g" % (k, out[k]))
    open(os.path.join(prof, tag + "_counters.md"), "w").write("\n".join(lines) + "\n")
    json.dump(out, open(os.path.join(prof, "prof_%s.json" % wl), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
