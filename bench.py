#!/usr/bin/env python3
"""Benchmark: aggregate Wasm instructions/sec of the batched MI355X interpreter.

Metric (BASELINE.json): "aggregate Wasm instrs/sec at 64K instances, 1/2/4/8 GPUs vs
host-core interp".  A step = one pass of the hot path over one batch: fresh instantiation
of 65,536 instances (memory image reset) + the interpreter kernel running every instance
to completion.  Instruction counts are the reference's Statistics counts
(include/common/statistics.h:44) produced per lane by the kernel itself.

Workload at N=1 (configs[1]): C2 -- 64K instances of the BLAKE3 compression loop
(wasmedge_amd/workloads.py), per-instance input.  Multi-GPU: one process per GPU
(torch.distributed.run), no data-path collective; a CPU-side (gloo) barrier +
max-over-ranks brackets the timed region.  The default is STRONG scaling, the metric's
configuration: the job's 64K instances (C5: 256K) split into contiguous id blocks over the
ranks ("scaling": "strong"); --scaling weak gives every rank 64K of its own.  At N > 1 the
line carries `expected_speedup` with its basis: 64K instances are 1024 waves, one per SIMD
of ONE GPU, so splitting them over more GPUs leaves SIMDs idle without shortening any
wave -- about 1x (C5's 4096 waves: up to 4x).

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
    if name == "c3grow":
        # not a BASELINE config: C3's sort in a module that starts with one page and
        # memory.grows to the pages the sort needs (the cost of growth)
        el = args.elements
        return (workloads.qsort_grow_wasm(), "sort", lambda ids: np.stack([ids, np.full_like(ids, el)], 1),
                [I32, I32], "C3 quicksort of %d i32 per instance, memory grown from 1 page by "
                            "memory.grow (no declared max)" % el, {"elements": el})
    if name == "c3x":
        # not a BASELINE config: C3's quicksort with its array on memory 1 (MultiMemories),
        # instruction for instruction C3's program on a memory past the first (VERDICT r5
        # item 8: the compiled XLD / XST against C3's memory-0 accesses)
        el = args.elements
        return (workloads.qsort_x_wasm(), "sort", lambda ids: np.stack([ids, np.full_like(ids, el)], 1),
                [I32, I32], "C3 quicksort of %d i32 per instance on memory 1 (MultiMemories)" % el,
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


SIMDS_PER_GPU = 256 * 4   # MI355X: 256 CUs x 4 SIMDs


def expected_speedup(total_instances, n_gpus, scaling):
    """What N GPUs can give over one on this job (reported, never measured here): a wave of
    64 instances runs on one SIMD, and its run time does not shrink when other SIMDs are
    idle (profiles/r02e_strong_scaling_c2.json: per-rank step time at 64K/N instances
    13.25 / 13.21 / 13.15 / 13.15 ms for N = 1/2/4/8 on one GPU). Strong scaling therefore
    speeds up only while one GPU holds more waves than SIMDs: min(N, waves / SIMDs), at
    least 1. Weak scaling: N (every GPU runs a whole job of its own)."""
    waves = -(-int(total_instances) // 64)
    if scaling == "weak":
        return {"value": float(n_gpus), "basis": "weak scaling: every GPU runs its own %d "
                "instances; instances are independent (no collective)" % (total_instances // n_gpus)}
    v = max(1.0, min(float(n_gpus), waves / SIMDS_PER_GPU))
    return {"value": v,
            "basis": "strong scaling: %d instances = %d waves of 64 against %d SIMDs per GPU; a "
                     "wave runs on one SIMD and its time does not shrink when other SIMDs idle, "
                     "so N GPUs give min(N, waves / SIMDs) = %.2fx (at least 1)"
                     % (total_instances, waves, SIMDS_PER_GPU, v)}


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


def cpu_baseline(wasm, func, build_rows, ptypes, budget_s, threads, gpu, what, tail_call=False,
                 multi_memory=False):
    """The oracle (C restatement of the reference interpreter, oracle/) timed on the
    box's host cores over a bounded sample of the same workload: chunks of instances
    (ids 0, 1, 2, ...), first on ONE thread for about budget_s / 4 seconds, then on
    `threads` threads for the rest of the budget (or until every instance ran). The
    oracle is the checker here too: the GPU's final state for the same instances must
    match bit for bit (status, return value, count, memory hash). Returns the baseline
    record, the sample's linear-memory bytes per wasm instruction, and those bytes split
    into (load, store) bytes per wasm instruction."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py
    m = oracle_py.Module(wasm, tail_call=tail_call, multi_memory=multi_memory)
    n_max = len(gpu["counts"])
    # chunks of about a quarter of a phase at the oracle's ~2e8 instr/s per thread
    t_inst = float(gpu["counts"].mean()) / 2e8
    rmask = 0xFFFFFFFF if gpu["ret32"] else 0xFFFFFFFFFFFFFFFF
    state = {"done": 0, "mbytes": 0.0, "sbytes": 0.0, "instrs": 0.0}

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
            state["sbytes"] += float(out["store_bytes"].sum())
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
    ld = (state["mbytes"] - state["sbytes"]) / state["instrs"]
    return rec, state["mbytes"] / state["instrs"], (ld, state["sbytes"] / state["instrs"])


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
    return args.workload in ("c3", "c3grow", "c3x") and args.elements >= 65536


# The job's instance count per workload when --instances is not given: the metric's "64K
# instances" (configs[1..3]) and C5's "256K across 8 MI355X" (configs[4]). With --gpus N > 1
# this is the FIXED TOTAL the ranks split (strong scaling, the metric's configuration);
# --scaling weak gives every rank that many instead.
DEFAULT_INSTANCES = {"c5": 262144}


def default_instances(workload):
    return DEFAULT_INSTANCES.get(workload, INSTANCES)


# Every bench workload runs on the compiled runs (DESIGN.md "Execution engines"): a context
# that reports none fell back to the threaded core (a hiprtc / assembly failure), and its
# line would silently measure a slower engine (the r04g failure mode).
def check_engine(workload, compiled_runs, engine, last_error=""):
    """SystemExit when a workload that compiles its runs in the test suite reports 0
    compiled runs (unless WB_JIT=0 asked for the interpreter)."""
    if compiled_runs == 0 and os.environ.get("WB_JIT", "1") != "0":
        raise SystemExit("bench.py: %s ran on %s with 0 compiled runs (silent fallback from the "
                         "compiled runs; last error: %s)" % (workload, engine, last_error or "none"))


def vary_ids(ids, step, workload):
    """Fresh inputs for step `step` (--vary-args): every instance gets another id -- a new
    tile, seed, block or start value -- shifted by a stride that is not a multiple of the
    wave size, so no wave sees the inputs of any earlier launch. C5's ids stay tile indices
    of the 4096^2 image (a permutation of its 262,144 tiles)."""
    shift = (step + 1) * 4099
    if workload == "c5":
        return (ids + shift) % 262144
    return (ids + shift) % (1 << 30)


class Phase:
    """One measured configuration: a context over `ids` (or over several devices), warmup,
    then exactly `steps` timed steps of Reset + Run. fresh: every step passes new arguments
    (vary_ids), uploaded before the step's clock starts -- the timed region is the same
    Reset + Run, on inputs the learned schedules have not seen."""

    def __init__(self, args, dist, ids, devices=None):
        from wasmedge_amd import batch
        self.args, self.dist, self.ids = args, dist, ids
        self.wasm, self.func, self.build_rows, self.ptypes, self.desc, self.extra = workload(args.workload, args)
        kw = {"max_memory_page": 17} if args.workload == "c3" else {}
        if args.workload == "tail":
            kw["tail_call"] = True
        if args.workload == "c3x":
            kw["multi_memory"] = True
        if args.cost_limit:
            kw["cost_limit"] = args.cost_limit
        if devices:
            kw["devices"] = devices
            kw["partition"] = batch.PARTITION_BLOCKS
        else:
            kw["device"] = dist.local_rank
        self.kw = kw
        self.batch = batch
        self.n = len(ids)
        self.values = batch.make_values(self.build_rows(ids), self.ptypes)
        self.t_start = time.perf_counter()
        self.t0 = time.perf_counter()
        self.ctx = batch.BatchContext(self.wasm, self.n, **kw)
        self.t_create = time.perf_counter() - self.t0
        self.e2e_s = {}

    def progress(self, msg):
        if self.dist.rank == 0:
            print("[bench] %s %.1fs" % (msg, time.perf_counter() - self.t_start), file=sys.stderr, flush=True)

    def outcome(self):
        _, st, cnt = self.ctx.results(1)
        traps = int((st != 0).sum())
        if traps and self.args.workload != "c4":
            raise SystemExit("%s instances trapped: %s" % (self.args.workload, np.unique(st)))
        return float(cnt.sum()), traps

    def warm(self, warmup):
        """End-to-end passes (SURVEY.md 8(d) variant ii), the warmup steps themselves:
         cold = BatchCreate (decode, validate, lower, hiprtc compile of the compiled runs,
                device allocation, instantiation) + SetArgs (params H2D) + Run + Results;
         warm = the same on the live context: SetArgs + Reset + Run + Results."""
        ctx = self.ctx
        t = self.t0
        ctx.set_args(self.func, self.values)
        self.instrs_per_step, self.traps = None, 0
        if warmup:
            ctx.run()
            self.instrs_per_step, self.traps = self.outcome()
            self.e2e_s["cold"] = time.perf_counter() - t
            self.progress("warmup 1/%d done (end-to-end cold)" % warmup)
        for w in range(1, warmup):
            t = time.perf_counter()
            ctx.set_args(self.func, self.values)
            ctx.reset()
            ctx.run()
            self.outcome()
            if w == 1:
                self.e2e_s["warm"] = time.perf_counter() - t
            self.progress("warmup %d/%d done" % (w + 1, warmup))
        check_engine(self.args.workload, ctx.compiled_runs(), ctx.engine(),
                     self.batch.lib().WasmEdge_BatchGetLastError(ctx._h).decode())

    def timed(self, steps):
        """Exactly `steps` timed steps bracketed by a barrier on both sides (BatchRun
        synchronises its stream); returns (max elapsed over ranks, kernel seconds)."""
        ctx, dist = self.ctx, self.dist
        dist.barrier()
        t0 = time.perf_counter()
        ksum = 0.0
        for k in range(steps):
            ctx.reset(timed=False)   # (no host round trip: the run orders after it)
            ksum += ctx.run()        # HIP-event time of the interpreter kernel (its stream)
            if elapsed_hint(self.args):
                self.progress("step %d/%d done" % (k + 1, steps))
        elapsed = time.perf_counter() - t0
        dist.barrier()
        if self.instrs_per_step is None:
            self.instrs_per_step, self.traps = self.outcome()
        _, st, cnt = ctx.results(1)
        assert float(cnt.sum()) == self.instrs_per_step and int((st != 0).sum()) == self.traps
        return dist.max(elapsed), ksum

    def fresh(self, steps):
        """--vary-args: `steps` steps, each on new arguments (vary_ids). SetArgs uploads them
        before the step's clock starts; the clock covers Reset + Run as in timed(). Returns
        (instructions, max over ranks of the summed step times, kernel seconds)."""
        ctx, dist = self.ctx, self.dist
        instrs, secs, ksum = 0.0, 0.0, 0.0
        for k in range(steps):
            vals = self.batch.make_values(self.build_rows(vary_ids(self.ids, k, self.args.workload)), self.ptypes)
            ctx.set_args(self.func, vals)
            dist.barrier()
            t0 = time.perf_counter()
            ctx.reset(timed=False)
            ksum += ctx.run()
            secs += time.perf_counter() - t0
            dist.barrier()
            _, st, cnt = ctx.results(1)
            if int((st != 0).sum()) and self.args.workload != "c4":
                raise SystemExit("fresh inputs: instances trapped: %s" % np.unique(st))
            instrs += float(cnt.sum())
        # (the repeated-input arguments again, for the hashes and checks after this)
        ctx.set_args(self.func, self.values)
        return dist.sum(instrs), dist.max(secs), ksum

    def close(self):
        self.ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong (default): --instances is the whole job's, split over the GPUs "
                         "(the metric's 64K instances; C5's 256K); weak: --instances per GPU")
    ap.add_argument("--no-weak", action="store_true",
                    help="with --gpus N > 1 and strong scaling: skip the extra weak-scaling phase")
    ap.add_argument("--in-process", action="store_true",
                    help="--gpus N from ONE process: one context over devices 0..N-1 "
                         "(WasmEdge_BatchConfigure::Devices) instead of a process per GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/rank plumbing only: shards, barrier and reductions, no GPU")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 20 for C2, whose step is ~1.6 ms; 3 otherwise)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 2 / 1)")
    ap.add_argument("--iters", type=int, default=ITERS)
    ap.add_argument("--instances", type=int, default=None,
                    help="instances (default 65536; 262144 for c5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c3grow", "c3x", "c4", "c5", "mt", "tail"])
    ap.add_argument("--mt-n", type=int, default=100000, help="mt19937 draws per instance")
    ap.add_argument("--elements", type=int, default=262144, help="C3 i32 per instance")
    ap.add_argument("--vary-args", default="auto", choices=["auto", "on", "off"],
                    help="also measure fresh inputs every step (the learned wave order and "
                         "layout never see them); auto = on for c5 and mt")
    ap.add_argument("--cost-limit", type=int, default=0,
                    help="meter gas with the unit cost table up to this limit (measures the "
                         "cost of exact metering; not the headline configuration)")
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 20 if args.workload == "c2" else 3
    if args.warmup is None:
        # (modules whose addresses may differ per instance run the layout trial over their
        # first three runs -- warm-up, 128-byte granules, 4-byte words: untimed)
        args.warmup = 2 if args.workload == "c2" else 3 if args.workload in ("c3", "c3grow", "c3x", "mt") else 1
    if args.instances is None:
        args.instances = default_instances(args.workload)
    if args.vary_args == "auto":
        args.vary_args = "on" if args.workload in ("c5", "mt") else "off"

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1 and not args.in_process:
        sys.exit(launch_workers(args.gpus, sys.argv[1:]))
    if world_env is not None and int(world_env) != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s" % (args.gpus, world_env))
    if args.in_process and world_env is not None and int(world_env) > 1:
        raise SystemExit("bench.py: --in-process runs one process, not one per GPU")
    dist = Dist()
    if args.dry_run:
        return dry_run(args, dist)
    n_gpus = args.gpus if args.in_process else dist.world
    devices = list(range(args.gpus)) if args.in_process and args.gpus > 1 else None
    # this rank's shard: the context holds exactly its instances (strong scaling splits
    # --instances over the ranks, weak gives every rank --instances of its own; in-process,
    # one context holds the whole job and the library splits it over the devices)
    ids = shard_ids(dist.rank, args.instances, dist.world, args.scaling)
    ph = Phase(args, dist, ids, devices)
    ph.warm(args.warmup)
    dist.init()
    elapsed, ksum = ph.timed(args.steps)
    instrs_per_step, traps, ctx, n = ph.instrs_per_step, ph.traps, ph.ctx, ph.n
    total_instrs = dist.sum(instrs_per_step) * args.steps
    # checksum of checksums over every instance's final linear memory (hash kernel, after
    # the timed region; before the fresh-input steps, which leave other instances' states)
    rets, st, cnt = ctx.results(1)
    hashes = ctx.memory_hash()
    fresh = None
    if args.vary_args == "on":
        fi, fs, fk = ph.fresh(args.steps)
        fresh = {"value": fi / fs, "ms_per_step": 1e3 * fs / args.steps,
                 "kernel_instr_per_s": fi / (dist.max(fk)),
                 "steps": args.steps,
                 "note": "every step on new arguments (instance i takes id (i + 4099*(k+1)) "
                         "mod %s): the wave order learned from earlier launches is keyed on "
                         "the arguments and is not reused; SetArgs before each step's clock, "
                         "the clock covers Reset + Run as for `value`"
                         % ("262144" if args.workload == "c5" else "2^30")}
    checksum = int(hashes.sum(dtype=np.uint64))
    gpu = {"counts": cnt, "hashes": hashes, "status": st, "ret": rets["lo"][:, 0],
           "ret32": args.workload not in ("c5", "mt")}
    kernel_avg = ksum / args.steps
    e2e = {"create_s": dist.max(ph.t_create)}
    for k in ("cold", "warm"):
        if k in ph.e2e_s:
            e2e["e2e_%s_s" % k] = dist.max(ph.e2e_s[k])
            e2e["e2e_%s_instr_per_s" % k] = dist.sum(instrs_per_step) / e2e["e2e_%s_s" % k]
    wasm, func, build_rows, ptypes, desc, extra = ph.wasm, ph.func, ph.build_rows, ph.ptypes, ph.desc, ph.extra
    if devices:
        par = "instance-sharded, 1 process over %d devices (WasmEdge_BatchConfigure::Devices, " \
              "contiguous wave blocks)" % len(devices)
    else:
        par = "instance-sharded, 1 process per GPU"
    out = {
        "metric": METRIC,
        "value": total_instrs / elapsed,
        "unit": "instr/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": {"c5": "f64", "mt": "i64"}.get(args.workload, "i32"),
        "data": "synthetic: per-instance inputs derived from the instance id inside the "
                "wasm module",
        "config": dict({"workload": desc, "instances_per_gpu": n // (len(devices) if devices else 1),
                        "instances": int(dist.sum(float(n))),
                        "instrs_per_instance": instrs_per_step / n,
                        "parallelism": par,
                        "compiled_runs": ctx.compiled_runs(), "engine": ctx.engine(),
                        "granule": ctx.memory_granule()}, **extra),
        "memory_checksum": "%016x" % checksum,
        "kernel_instr_per_s": total_instrs / (dist.max(kernel_avg) * args.steps),
        # the interpreter kernel's mean duration per step, HIP events on the library's stream
        # (the rooflines' time basis); ms_per_step adds the Reset and the launch gaps
        "kernel_ms": 1e3 * dist.max(kernel_avg),
    }
    if fresh:
        out["fresh_input"] = fresh
    if args.workload == "c4":
        out["config"]["trapped_instances"] = traps
    if args.cost_limit:
        out["config"]["cost_limit"] = args.cost_limit
    c3_bytes_per_instr, c3_bpi_src = C3_BYTES_PER_INSTR, ", committed oracle figure"
    c3_split = None
    if dist.rank == 0 and dist.world == 1 and not devices and not args.no_cpu_baseline:
        threads = host_cores()
        out["cpu_baseline"], bpi, c3_split = cpu_baseline(wasm, func, build_rows, ptypes, args.cpu_seconds,
                                                          threads, gpu, args.workload.upper(),
                                                          tail_call=args.workload == "tail",
                                                          multi_memory=args.workload == "c3x")
        if args.workload in ("c3", "c3grow", "c3x"):
            # qsort's bytes per instruction is stable across instances
            c3_bytes_per_instr, c3_bpi_src = bpi, " on the oracle sample"
    if args.workload != "c2":
        out["data"] = "synthetic: per-instance inputs derived from the instance id"
    out["workload_key"] = args.workload
    out.update(e2e)
    prof = load_profile(args.workload, out["config"])
    kernel_max = dist.max(kernel_avg)
    rooflines(out, args, prof, instrs_per_step, kernel_max, n, c3_bytes_per_instr, c3_bpi_src, c3_split)
    ph.close()
    # the metric's configuration at N > 1 is the fixed total (strong); the weak-scaling
    # figure (every rank --instances of its own) rides along as an extra key
    if n_gpus > 1:
        out["expected_speedup"] = expected_speedup(out["config"]["instances"], n_gpus, args.scaling)
    if n_gpus > 1 and args.scaling == "strong" and not args.no_weak:
        wids = shard_ids(dist.rank, args.instances, dist.world, "weak") if not devices else \
            np.arange(args.instances * len(devices), dtype=np.int64)
        wp = Phase(args, dist, wids, devices)
        wp.warm(1)
        we, _ = wp.timed(args.steps)
        wi = dist.sum(wp.instrs_per_step) * args.steps
        out["weak_scaling"] = {"value": wi / we, "ms_per_step": 1e3 * we / args.steps,
                               "instances": int(dist.sum(float(len(wids)))),
                               "instances_per_gpu": args.instances,
                               "note": "every GPU runs --instances of its own (ids disjoint)"}
        wp.close()
    if dist.rank == 0:
        print(json.dumps(out), flush=True)


def rooflines(out, args, prof, instrs_per_step, kernel_max, n, c3_bytes_per_instr, c3_bpi_src, c3_split):
    traffic = prof.get("hbm_bytes_per_launch")
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
    # one time basis, named: `achieved` / `frac` use this run's HIP-event kernel time; the
    # profile's traced kernel time (rocprofv3 kernel trace of the same command, another run)
    # gives `frac_traced`, and the profile also records the HIP-event time its own bench run
    # measured, so the two clocks can be compared in the same process
    timing = {"time_basis": "kernel_ms: this run's HIP-event kernel time on the library's stream",
              "kernel_ms": 1e3 * kernel_max}
    if prof.get("kernel_avg_ns"):
        timing["traced_kernel_ms"] = prof["kernel_avg_ns"] / 1e6
        if prof.get("bench_kernel_ms"):
            timing["traced_run_hip_event_kernel_ms"] = prof["bench_kernel_ms"]
        if timing["traced_kernel_ms"] > out["ms_per_step"]:
            timing["note"] = ("the traced kernel (%.4g ms, rocprofv3 kernel trace of another run%s) is "
                              "longer than this line's step (%.4g ms): the trace pass runs under the "
                              "profiler on another box; frac uses this run's own kernel time"
                              % (timing["traced_kernel_ms"],
                                 ", whose own HIP events read %.4g ms" % prof["bench_kernel_ms"]
                                 if prof.get("bench_kernel_ms") else "", out["ms_per_step"]))
    if prof.get("valu_insts_per_launch"):
        valu = prof["valu_insts_per_launch"] * 64.0 / kernel_max
        wps = prof.get("waves_per_simd")
        issue.update(timing)
        if prof.get("kernel_avg_ns"):
            issue["frac_traced"] = prof["valu_insts_per_launch"] * 64.0 / (prof["kernel_avg_ns"] * 1e-9) / VALU_PEAK
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
    if args.workload in ("c3", "c3grow", "c3x"):
        # HBM-bound config: algorithmic bytes = the linear-memory bytes of the wasm loads and
        # stores, per wasm instruction as the oracle counts them on the CPU-baseline sample
        # (or the committed figure when the baseline leg is skipped) x this launch's count
        bpi = c3_bytes_per_instr
        bytes_launch = bpi * instrs_per_step
        achieved = bytes_launch / kernel_max / 1e9
        out["roofline"] = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                           "traffic": traffic, **timing,
                           "note": "algorithmic = linear-memory bytes of the wasm loads and "
                                   "stores (%.4f B per wasm instr%s); traffic = HBM bytes per "
                                   "launch, FETCH_SIZE x 2 (MI355X_MICROARCH.md 'HBM') + "
                                   "WRITE_SIZE" % (bpi, c3_bpi_src)}
        if c3_split:
            ld, stb = c3_split
            out["roofline"]["algorithmic_load_bytes"] = ld * instrs_per_step
            out["roofline"]["algorithmic_store_bytes"] = stb * instrs_per_step
        if prof.get("write_bytes") and c3_split:
            out["roofline"]["write_over_store_bytes"] = prof["write_bytes"] / (c3_split[1] * instrs_per_step)
        if prof.get("kernel_avg_ns"):
            out["roofline"]["frac_traced"] = bytes_launch / (prof["kernel_avg_ns"] * 1e-9) / 1e9 / HBM_PEAK_GBS
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
        line = {"dry_run": True, "n_gpus": dist.world, "scaling": args.scaling,
                "instances": int(total), "first_id": int(lo), "last_id": int(hi),
                "max_over_ranks": t}
        if dist.world > 1:
            line["expected_speedup"] = expected_speedup(int(total), dist.world, args.scaling)
        print(json.dumps(line), flush=True)
    if dist.td:
        dist.td.destroy_process_group()
    return 0


if __name__ == "__main__":
    main()
