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


def cpu_baseline(wasm, func, build_rows, ptypes, budget_s, threads, gpu, what):
    """The oracle (C restatement of the reference interpreter, oracle/) timed on the
    box's host cores over a bounded sample of the same workload: chunks of instances
    (ids 0, 1, 2, ...), first on ONE thread for about budget_s / 4 seconds, then on
    `threads` threads for the rest of the budget (or until every instance ran). The
    oracle is the checker here too: the GPU's final state for the same instances must
    match bit for bit (status, return value, count, memory hash). Returns the baseline
    record and the sample's linear-memory bytes per wasm instruction."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    m = oracle_py.Module(wasm)
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
                          "time on fib(30) and 3.5x on mt19937 (BASELINE.md 3)"}
    return rec, state["mbytes"] / state["instrs"]


def load_profile():
    """The committed rocprofv3 PMC summary of this bench command (profiles/traffic_c2.json,
    tools/prof_summary.py): HBM bytes and VALU instructions per interpreter launch, when
    it matches the configuration (see DESIGN.md 'Measurement')."""
    p = os.path.join(ROOT, "profiles", "traffic_c2.json")
    if os.path.exists(p):
        with open(p) as f:
            d = json.load(f)
        if d.get("iters") == ITERS and d.get("instances") == INSTANCES:
            return d
    return {}


def load_profile_traffic():
    return load_profile().get("hbm_bytes_per_launch")


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
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c4", "c5"])
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
    n = args.instances
    kw = {"max_memory_page": 17} if args.workload == "c3" else {}
    if args.cost_limit:
        kw["cost_limit"] = args.cost_limit
    ctx = batch.BatchContext(wasm, n, device=dist.local_rank, **kw)
    ids = shard_ids(dist.rank, n, dist.world, args.scaling)
    n = len(ids)
    rows = build_rows(ids)
    ctx.set_args(func, batch.make_values(rows, ptypes))
    nret = 1
    dist.init()

    def progress(msg):
        if dist.rank == 0:
            print("[bench] %s %.1fs" % (msg, time.perf_counter() - t_start), file=sys.stderr, flush=True)

    t_start = time.perf_counter()
    for w in range(args.warmup):
        ctx.reset()
        ctx.run()
        progress("warmup %d/%d done" % (w + 1, args.warmup))
    _, st, cnt = ctx.results(nret)
    traps = int((st != 0).sum())
    if traps and args.workload != "c4":
        raise SystemExit("%s instances trapped: %s" % (args.workload, np.unique(st)))
    instrs_per_step = float(cnt.sum())

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
    total_instrs = dist.sum(instrs_per_step) * args.steps
    rets, st, cnt = ctx.results(nret)
    assert float(cnt.sum()) == instrs_per_step and int((st != 0).sum()) == traps
    # checksum of checksums over every instance's final linear memory (hash kernel, after
    # the timed region)
    hashes = ctx.memory_hash()
    checksum = int(hashes.sum(dtype=np.uint64))
    gpu = {"counts": cnt, "hashes": hashes, "status": st, "ret": rets["lo"][:, 0],
           "ret32": args.workload != "c5"}
    kernel_avg = ksum / args.steps
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
        "dtype": "i32" if args.workload != "c5" else "f64",
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
    if args.workload == "c2":
        bytes_launch = float(c2_mem_bytes(args.iters)) * n
        achieved = bytes_launch / kernel_avg / 1e9
        out["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                           "traffic": load_profile_traffic(),
                           "note": "algorithmic = linear-memory bytes the wasm program moves; "
                                   "the path is dispatch-issue bound, see issue_roofline"}

    else:
        out["data"] = "synthetic: per-instance inputs derived from the instance id"
    # the bound that matters for the interpreter: vector issue at one wave per SIMD. The
    # achieved rate is the VALU lane-ops the kernel issues (SQ_INSTS_VALU x 64 from the
    # committed PMC pass of this same command) over this run's measured kernel time
    per_gpu = total_instrs / elapsed / dist.world
    prof = load_profile() if (args.workload == "c2" and args.iters == ITERS and n == INSTANCES) else {}
    if prof.get("valu_insts_per_launch"):
        valu = prof["valu_insts_per_launch"] * 64.0 / kernel_avg
        out["issue_roofline"] = {
            "bound": "valu", "achieved": valu, "peak": VALU_PEAK, "unit": "VALU lane-op/s",
            "frac": valu / VALU_PEAK,
            "wasm_instr_per_valu_lane_op": (total_instrs / args.steps / dist.world) /
                                           (prof["valu_insts_per_launch"] * 64.0),
            "source": "SQ_INSTS_VALU per launch, profiles/%s_counters.md" % prof.get("source"),
            "basis": "DESIGN.md 'Roofline': 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz "
                     "(MI355X_MICROARCH.md)"}
    else:
        out["issue_roofline"] = {
            "bound": "valu", "achieved": None, "peak": VALU_PEAK, "unit": "VALU lane-op/s",
            "frac": None, "wasm_instr_per_s_per_gpu": per_gpu,
            "note": "no PMC summary for this configuration (tools/prof_bench.sh)"}
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        threads = host_cores()
        out["cpu_baseline"], bpi = cpu_baseline(wasm, func, build_rows, ptypes, args.cpu_seconds,
                                                threads, gpu, args.workload.upper())
        if args.workload == "c3":
            # algorithmic bytes: the linear-memory bytes the wasm program moves, counted
            # per instance by the oracle on the sample, per instruction x this launch's
            # instructions (qsort's bytes per instruction is stable across instances)
            bytes_launch = bpi * instrs_per_step
            achieved = bytes_launch / kernel_avg / 1e9
            out["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                               "note": "algorithmic = linear-memory bytes of the wasm loads and "
                                       "stores (%.3f B per wasm instr on the oracle sample)" % bpi}
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
