#!/usr/bin/env python3
"""Benchmark: aggregate Wasm instructions/sec of the batched MI355X interpreter.

Metric (BASELINE.json): "aggregate Wasm instrs/sec at 64K instances, 1/2/4/8 GPUs vs
host-core interp".  A step = one pass of the hot path over one batch: fresh instantiation
of 65,536 instances (memory image reset) + the interpreter kernel running every instance
to completion.  Instruction counts are the reference's Statistics counts
(include/common/statistics.h:44) produced per lane by the kernel itself.

Workload at N=1 (configs[1]): C2 -- 64K instances of the BLAKE3 compression loop
(wasmedge_amd/workloads.py), per-instance input.  Multi-GPU: one process per GPU
(torch.distributed.run), each rank runs its own 64K-instance shard (instance ids
[rank*64K, (rank+1)*64K)), no data-path collective -> "scaling": "weak"; a CPU-side
(gloo) barrier + max-over-ranks brackets the timed region.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "aggregate Wasm instrs/sec at 64K instances, 1/2/4/8 GPUs vs host-core interp"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip-level parameters
VALU_PEAK = 256 * 4 * 32 * 2.4e9   # VALU lane-ops/s: 256 CUs x 4 SIMD-32 x 2.4 GHz
INSTANCES = 65536
ITERS = 1000                   # chained compressions per instance
# C3 linear-memory bytes per wasm instruction, counted by the oracle over CPU-baseline
# samples of 262,144-element sorts (r02/r03 bench lines: 0.410); used when the baseline leg
# is skipped (profiling runs)
C3_BYTES_PER_INSTR = 0.4100


def c2_mem_bytes(iters):
    """Algorithmic linear-memory bytes of one C2 instance: 12 x i64.store fill (96 B),
    per compression 16+8 i32.load + 8 i32.store (128 B), final i32.load (4 B)."""
    return 96 + 128 * iters + 4


def workload(name, args):
    """(wasm, export, rows builder(ids) -> int64[n, k], param types, description) of a
    BASELINE.json config. The default bench line is C2 (configs[1]); the others are
    selectable with --workload for the per-config numbers in DESIGN.md."""
    from wasmedge_amd import batch, workloads
    I32 = batch.I32
    if name == "c2":
        it = args.iters
        return (workloads.blake3_wasm(), "run", lambda ids: np.stack([ids, np.full_like(ids, it)], 1),
                [I32, I32], "C2 BLAKE3 compression loop (configs[1])", {"iters": it})
    if name == "c1":
        fib = open(os.path.join(ROOT, "tests", "golden", "fibonacci.wasm"), "rb").read()
        return (fib, "fib", lambda ids: (20 + ids % 11)[:, None], [I32],
                "C1 recursive fib(n), n = 20 + id mod 11 (configs[0] on the GPU)", {})
    if name == "c3":
        el = args.elements
        return (workloads.qsort_wasm(), "sort", lambda ids: np.stack([ids, np.full_like(ids, el)], 1),
                [I32, I32], "C3 quicksort of %d i32 per instance (configs[2])" % el,
                {"elements": el})
    if name == "c4":
        return (workloads.collatz_wasm(), "collatz",
                lambda ids: np.stack([ids, np.full_like(ids, 10000)], 1), [I32, I32],
                "C4 Collatz br_table state machine + per-lane traps (configs[3])", {})
    if name == "c5":
        return (workloads.mandel_wasm(), "tile",
                lambda ids: np.stack([ids, np.full_like(ids, 4096), np.full_like(ids, 50)], 1),
                [I32, I32, I32], "C5 f64x2 Mandelbrot 8x8 tiles of 4096^2, 50 iters (configs[4])",
                {})
    if name == "mt":
        # not a BASELINE config: a second real module through the compiled runs (VERDICT r2
        # item 8) -- the reference's own mt19937 test module (i64 + SIMD128 + memory),
        # every instance drawing `mt_n` numbers from its own seed
        mt = open(os.path.join(ROOT, "tests", "golden", "mt19937.wasm"), "rb").read()
        n = args.mt_n
        return (mt, "mt19937",
                lambda ids: np.stack([np.zeros_like(ids), 5489 + ids, np.full_like(ids, n)], 1),
                [batch.I32, batch.I64, batch.I64],
                "mt19937 of test/thread/ThreadTest.cpp:31-163, %d draws from a per-instance seed" % n,
                {"draws": n})
    if name == "tail":
        # not a BASELINE config: the TailCall proposal's return_call / return_call_indirect
        # (tail recursion, mutual recursion through a table), 5000 + id mod 13 outer steps
        return (workloads.tail_wasm(), "run",
                lambda ids: np.stack([ids, np.full_like(ids, 5000)], 1), [I32, I32],
                "tail-recursive countdown + mutual even/odd (return_call, return_call_indirect)",
                {"steps": 5000})
    raise SystemExit("unknown workload " + name)


class Dist:
    """Barrier + max over ranks. torch.distributed (gloo, CPU-side) only when
    WORLD_SIZE > 1, imported after the HIP library so the two HIP runtimes never mix
    on the GPU."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.td = None

    def init(self):
        if self.world > 1:
            import torch.distributed as td
            td.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.td = td

    def barrier(self):
        if self.td:
            self.td.barrier()

    def max(self, x):
        if not self.td:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.td.all_reduce(t, op=self.td.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if not self.td:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.td.all_reduce(t, op=self.td.ReduceOp.SUM)
        return float(t.item())


def shard_ids(rank, n, world=1, scaling="weak"):
    """Instance ids of this rank's shard. weak: [rank*n, (rank+1)*n) -- every rank runs n
    instances of its own, N GPUs process N*n distinct instances. strong: the n instances
    of the job split into contiguous blocks, [rank*n/N, (rank+1)*n/N)."""
    if scaling == "strong":
        lo, hi = rank * n // world, (rank + 1) * n // world
        return np.arange(lo, hi, dtype=np.int64)
    return np.arange(rank * n, (rank + 1) * n, dtype=np.int64)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_workers(n, argv):
    """`bench.py --gpus N` run directly (not under torch.distributed.run): start N worker
    processes of this script, one per GPU (RANK = LOCAL_RANK = r, 127.0.0.1 rendezvous),
    wait for all of them and return the worst exit status. This parent never touches the
    GPU (no HIP call, no torch.cuda) and never execs; rank 0 prints the JSON line."""
    import subprocess
    env = dict(os.environ)
    env.update(WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=env.get("MASTER_PORT") or str(_free_port()))
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def host_cores():
    """Host threads for the CPU baseline: the CPUs this process may run on, capped at 16
    (the GPU box's CPU share per GPU; os.cpu_count() there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(wasm, func, build_rows, ptypes, budget_s, threads, gpu, what, tail_call=False):
    """The oracle (C restatement of the reference interpreter, oracle/) timed on the
    box's host cores over a bounded sample of the same workload: chunks of instances
    (ids 0, 1, 2, ...), first on ONE thread for about budget_s / 4 seconds, then on
    `threads` threads for the rest of the budget (or until every instance ran). The
    oracle is the checker here too: the GPU's final state for the same instances must
    match bit for bit (status, return value, count, memory hash). Returns the baseline
    record and the sample's linear-memory bytes per wasm instruction."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    m = oracle_py.Module(wasm, tail_call=tail_call)
    n_max = len(gpu["counts"])
    # chunks of about a quarter of a phase at the oracle's ~2e8 instr/s per thread
    t_inst = float(gpu["counts"].mean()) / 2e8
    rmask = 0xFFFFFFFF if gpu["ret32"] else 0xFFFFFFFFFFFFFFFF
    state = {"done": 0, "mbytes": 0.0, "instrs": 0.0}

    def phase(nthr, budget):
        # ids wrap round: a phase that runs out of instances starts over (checked again)
        chunk = int(max(nthr, min(64 * nthr, nthr * budget / 4 / max(t_inst, 1e-9))))
        instrs, secs, ran = 0.0, 0.0, 0
        while secs < budget and (nthr > 1 or ran < n_max):
            k = min(chunk, n_max)
            ids = (state["done"] + np.arange(k, dtype=np.int64)) % n_max
            rows = build_rows(ids)
            params = np.zeros((k, len(ptypes), 2), np.uint64)
            params[:, :, 0] = rows.astype(np.uint64)
            out = m.run_batch(func, params, k, threads=nthr)
            if not (np.array_equal(out["codes"], gpu["status"][ids])
                    and np.array_equal(out["counts"], gpu["counts"][ids])
                    and np.array_equal(out["hashes"], gpu["hashes"][ids])
                    and np.array_equal((out["results"][:, 0, 0] & rmask)[out["codes"] == 0],
                                       (gpu["ret"][ids] & rmask)[out["codes"] == 0])):
                raise SystemExit("GPU/oracle mismatch in instances %d..%d" % (ids[0], ids[-1]))
            instrs += float(out["counts"].sum())
            state["mbytes"] += float(out["mem_bytes"].sum())
            secs += out["seconds"]
            state["done"] = int((ids[-1] + 1) % n_max)
            ran += k
        state["instrs"] += instrs
        return instrs, secs, ran

    i1, s1, n1 = phase(1, budget_s / 4)
    it, st, nt = phase(threads, budget_s - s1)
    rec = {"value": it / st, "unit": "instr/s", "cores": threads, "kind": "port",
           "value_1thread": i1 / s1, "cpu_model": cpu_model(),
           "sample": "%s instances: %d on 1 thread (%.3g instrs, %.2fs), then %d on %d threads "
                     "(%.3g instrs, %.2fs), ids from 0 wrapping round; all bit-exact vs the GPU run "
                     "on those instances"
                     % (what, n1, i1, s1, nt, threads, it, st),
           "calibration": "the oracle on 1 thread takes 0.9-1.4x the reference interpreter's "
                          "time on fib(30) and 2-2.5x on mt19937 (BASELINE.md 3)"}
    return rec, state["mbytes"] / state["instrs"]


def load_profile(workload, config):
    """The committed rocprofv3 summary of this bench configuration
    (profiles/prof_<workload>.json, written by tools/prof_summary.py from a
    tools/prof_bench.sh run of the same command): HBM bytes, VALU instructions, active
    lanes per VALU instruction, resident waves per SIMD, VMEM latency per interpreter
    launch -- only when its configuration equals this run's (DESIGN.md 'Measurement')."""
    p = os.path.join(ROOT, "profiles", "prof_%s.json" % workload)
    if not os.path.exists(p):
        return {}
    with open(p) as f:
        d = json.load(f)
    key = {k: config[k] for k in ("workload", "instances_per_gpu", "elements", "iters", "draws") if k in config}
    return d if {k: v for k, v in d.get("config", {}).items() if v is not None} == key else {}


def elapsed_hint(args):
    """Long steps (full-size C3) report progress on stderr so a run is never silent for
    minutes; short ones stay quiet inside the timed region."""
    return args.workload == "c3" and args.elements >= 65536


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: --instances per GPU; strong: --instances for the whole job")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rank plumbing only: shards, barrier and reductions, no GPU")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 20 for C2, whose step is ~1.6 ms; 3 otherwise)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 2 / 1)")
    ap.add_argument("--iters", type=int, default=ITERS)
    ap.add_argument("--instances", type=int, default=INSTANCES)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "mt", "tail"])
    ap.add_argument("--mt-n", type=int, default=100000, help="mt19937 draws per instance")
    ap.add_argument("--elements", type=int, default=262144, help="C3 i32 per instance")
    ap.add_argument("--cost-limit", type=int, default=0,
                    help="meter gas with the unit cost table up to this limit (measures the "
                         "cost of exact metering; not the headline configuration)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 20 if args.workload == "c2" else 3
    if args.warmup is None:
        args.warmup = 2 if args.workload == "c2" else 1

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_workers(args.gpus, sys.argv[1:]))
    if world_env is not None and int(world_env) != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s" % (args.gpus, world_env))
    dist = Dist()
    if args.dry_run:
        return dry_run(args, dist)
    from wasmedge_amd import batch
    wasm, func, build_rows, ptypes, desc, extra = workload(args.workload, args)
    # this rank's shard first: the context holds exactly its instances (strong scaling
    # splits --instances over the ranks, weak gives every rank --instances of its own)
    ids = shard_ids(dist.rank, args.instances, dist.world, args.scaling)
    n = len(ids)
    kw = {"max_memory_page": 17} if args.workload == "c3" else {}
    if args.workload == "tail":
        kw["tail_call"] = True
    if args.cost_limit:
        kw["cost_limit"] = args.cost_limit
    rows = build_rows(ids)
    values = batch.make_values(rows, ptypes)
    nret = 1
    t_start = time.perf_counter()

    def progress(msg):
        if dist.rank == 0:
            print("[bench] %s %.1fs" % (msg, time.perf_counter() - t_start), file=sys.stderr, flush=True)

    def outcome():
        _, st, cnt = ctx.results(nret)
        traps = int((st != 0).sum())
        if traps and args.workload != "c4":
            raise SystemExit("%s instances trapped: %s" % (args.workload, np.unique(st)))
        return float(cnt.sum()), traps

    # End-to-end passes (SURVEY.md 8(d) variant ii), the warmup steps themselves:
    #  cold = BatchCreate (decode, validate, lower, hiprtc compile of the compiled runs,
    #         device allocation, instantiation) + SetArgs (params H2D) + Run + Results
    #         (returns, statuses, counts D2H);
    #  warm = the same on the live context: SetArgs + Reset + Run + Results.
    t = time.perf_counter()
    ctx = batch.BatchContext(wasm, n, device=dist.local_rank, **kw)
    t_create = time.perf_counter() - t
    ctx.set_args(func, values)
    e2e_s = {}
    if args.warmup:
        ctx.run()
        instrs_per_step, traps = outcome()
        e2e_s["cold"] = time.perf_counter() - t
        progress("warmup 1/%d done (end-to-end cold)" % args.warmup)
    for w in range(1, args.warmup):
        t = time.perf_counter()
        ctx.set_args(func, values)
        ctx.reset()
        ctx.run()
        outcome()
        if w == 1:
            e2e_s["warm"] = time.perf_counter() - t
        progress("warmup %d/%d done" % (w + 1, args.warmup))
    dist.init()

    dist.barrier()
    t0 = time.perf_counter()
    ksum = 0.0
    for k in range(args.steps):
        ctx.reset(timed=False)   # (no host round trip: the run orders after it)
        ksum += ctx.run()        # HIP-event time of the interpreter kernel (its stream)
        if elapsed_hint(args):
            progress("step %d/%d done" % (k + 1, args.steps))
    elapsed = time.perf_counter() - t0   # BatchRun synchronises its stream
    dist.barrier()
    elapsed = dist.max(elapsed)
    if not args.warmup:
        instrs_per_step, traps = outcome()
    rets, st, cnt = ctx.results(nret)
    assert float(cnt.sum()) == instrs_per_step and int((st != 0).sum()) == traps
    total_instrs = dist.sum(instrs_per_step) * args.steps
    # checksum of checksums over every instance's final linear memory (hash kernel, after
    # the timed region)
    hashes = ctx.memory_hash()
    checksum = int(hashes.sum(dtype=np.uint64))
    gpu = {"counts": cnt, "hashes": hashes, "status": st, "ret": rets["lo"][:, 0],
           "ret32": args.workload not in ("c5", "mt")}
    kernel_avg = ksum / args.steps
    e2e = {"create_s": dist.max(t_create)}
    for k in ("cold", "warm"):
        if k in e2e_s:
            e2e["e2e_%s_s" % k] = dist.max(e2e_s[k])
            e2e["e2e_%s_instr_per_s" % k] = dist.sum(instrs_per_step) / e2e["e2e_%s_s" % k]
    out = {
        "metric": METRIC,
        "value": total_instrs / elapsed,
        "unit": "instr/s",
        "n_gpus": dist.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": {"c5": "f64", "mt": "i64"}.get(args.workload, "i32"),
        "data": "synthetic: per-instance inputs derived from the instance id inside the "
                "wasm module",
        "config": dict({"workload": desc, "instances_per_gpu": n,
                        "instances": int(dist.sum(float(n))),
                        "instrs_per_instance": instrs_per_step / n,
                        "parallelism": "instance-sharded, 1 process per GPU"}, **extra),
        "memory_checksum": "%016x" % checksum,
        "kernel_instr_per_s": total_instrs / (dist.max(kernel_avg) * args.steps),
    }
    if args.workload == "c4":
        out["config"]["trapped_instances"] = traps
    if args.cost_limit:
        out["config"]["cost_limit"] = args.cost_limit
    c3_bytes_per_instr, c3_bpi_src = C3_BYTES_PER_INSTR, ", committed oracle figure"
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        threads = host_cores()
        out["cpu_baseline"], bpi = cpu_baseline(wasm, func, build_rows, ptypes, args.cpu_seconds,
                                                threads, gpu, args.workload.upper(),
                                                tail_call=args.workload == "tail")
        if args.workload == "c3":
            # qsort's bytes per instruction is stable across instances
            c3_bytes_per_instr, c3_bpi_src = bpi, " on the oracle sample"
    if args.workload != "c2":
        out["data"] = "synthetic: per-instance inputs derived from the instance id"
    out["workload_key"] = args.workload
    out.update(e2e)
    prof = load_profile(args.workload, out["config"])
    kernel_max = dist.max(kernel_avg)
    # The interpreter's bound is vector issue (VALU), not HBM, for every config but C3:
    # SQ_INSTS_VALU per launch (committed PMC pass of this same command) x 64 lanes over
    # this run's live kernel time (HIP events on the library's stream), against 256 CU x
    # 4 SIMD-32 x 32 lanes x 2.4 GHz. One wave alone issues a VALU instruction every 4
    # cycles at best, so at one wave per SIMD (64K instances) 0.5 of that peak is the
    # ceiling (2 waves per SIMD: 1.0).
    issue = {"bound": "valu", "achieved": None, "peak": VALU_PEAK, "unit": "VALU lane-op/s",
             "frac": None,
             "basis": "256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md); one "
                      "wave issues VALU at most every 4 cycles"}
    if prof.get("valu_insts_per_launch"):
        valu = prof["valu_insts_per_launch"] * 64.0 / kernel_max
        wps = prof.get("waves_per_simd")
        issue.update({
            "achieved": valu, "frac": valu / VALU_PEAK,
            "single_wave_ceiling": min(1.0, 0.5 * wps) if wps else None,
            "waves_per_simd": wps,
            "lanes_per_valu": prof.get("lanes_per_valu"),
            "wasm_instr_per_valu_lane_op": instrs_per_step / (prof["valu_insts_per_launch"] * 64.0),
            "source": "profiles/%s_counters.md (SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU, "
                      "SQ_WAVE_CYCLES per launch)" % prof.get("source")})
    else:
        issue["note"] = "no PMC summary for this configuration (tools/prof_bench.sh)"
    traffic = prof.get("hbm_bytes_per_launch")
    if args.workload == "c3":
        # HBM-bound config: algorithmic bytes = the linear-memory bytes of the wasm loads and
        # stores, per wasm instruction as the oracle counts them on the CPU-baseline sample
        # (or the committed figure when the baseline leg is skipped) x this launch's count
        bpi = c3_bytes_per_instr
        bytes_launch = bpi * instrs_per_step
        achieved = bytes_launch / kernel_max / 1e9
        out["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                           "traffic": traffic,
                           "note": "algorithmic = linear-memory bytes of the wasm loads and "
                                   "stores (%.4f B per wasm instr%s); traffic = HBM bytes per "
                                   "launch from FETCH_SIZE + WRITE_SIZE" % (bpi, c3_bpi_src)}
        out["issue_roofline"] = issue
    else:
        out["roofline"] = dict(issue)
        hbm = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": traffic,
               "achieved": traffic / kernel_max / 1e9 if traffic else None}
        if hbm["achieved"] is not None:
            hbm["frac"] = hbm["achieved"] / HBM_PEAK_GBS
        if args.workload == "c2":
            hbm["wasm_level_bytes"] = float(c2_mem_bytes(args.iters)) * n
            hbm["note"] = ("the wasm program names %.4g B of linear memory per launch, but the "
                           "compiled loop forwards its loads in registers: the counters see the "
                           "stores only" % hbm["wasm_level_bytes"])
        out["hbm_roofline"] = hbm
    if dist.rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()


def dry_run(args, dist):
    """The multi-process plumbing without a GPU: each rank takes its shard, joins the
    barrier and the max/sum reductions exactly as a measured run does; rank 0 prints the
    resulting layout as the JSON line (no metric value)."""
    dist.init()
    ids = shard_ids(dist.rank, args.instances, dist.world, args.scaling)
    dist.barrier()
    t = dist.max(float(dist.rank + 1))
    total = dist.sum(float(len(ids)))
    lo = dist.sum(float(ids[0]) if dist.rank == 0 else 0.0)
    hi = dist.max(float(ids[-1]))
    dist.barrier()
    if dist.rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": dist.world, "scaling": args.scaling,
                          "instances": int(total), "first_id": int(lo), "last_id": int(hi),
                          "max_over_ranks": t}), flush=True)
    if dist.td:
        dist.td.destroy_process_group()
    return 0


if __name__ == "__main__":
    main()
