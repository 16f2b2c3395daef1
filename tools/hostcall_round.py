"""Time one host-call service round at 64K lanes (DESIGN.md "Host
imports"): every instance writes a 24-byte line to stdout through WASI fd_write once, so
the launch parks all 65,536 lanes, the host serves them in one round (hostcall.cpp:
bulk copies + per-wave memory blocks on a thread pool) and the kernel resumes them.
Prints a JSON line: BatchRun wall time with the call, without it (same module, the call
skipped by its argument), their difference = the round, per lane; the captured output of
a few instances is checked. Tuning aid, not a test: python tools/hostcall_round.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from wasmedge_amd import batch  # noqa: E402
from wasmedge_amd.wat import assemble  # noqa: E402

WASM = assemble(r"""
(module
  (import "wasi_snapshot_preview1" "fd_write" (func $fd_write (param i32 i32 i32 i32) (result i32)))
  (memory 1)
  (data (i32.const 1024) "instance output line 00\n")
  (func (export "run") (param $id i32) (param $call i32) (result i32)
    ;; per-instance digits at 1044, iovec at 2048, nwritten at 2100
    (i32.store8 (i32.const 1045) (i32.add (i32.const 48) (i32.rem_u (i32.div_u (local.get $id) (i32.const 10)) (i32.const 10))))
    (i32.store8 (i32.const 1046) (i32.add (i32.const 48) (i32.rem_u (local.get $id) (i32.const 10))))
    (i32.store (i32.const 2048) (i32.const 1024))
    (i32.store (i32.const 2052) (i32.const 24))
    (if (result i32) (local.get $call)
      (then (call $fd_write (i32.const 1) (i32.const 2048) (i32.const 1) (i32.const 2100)))
      (else (i32.const 0)))))
""")


def timed(call, n, threads, reps=3):
    ctx = batch.BatchContext(WASM, n, host_threads=threads)
    try:
        ctx.init_wasi()
        vals = batch.make_values([[i, call] for i in range(n)], [batch.I32, batch.I32])
        best = 1e9
        for _ in range(reps):
            ctx.init_wasi()           # clears the captured output
            ctx.reset()
            ctx.set_args("run", vals)
            t = time.perf_counter()
            ctx.run()
            best = min(best, time.perf_counter() - t)
        _, st, _ = ctx.results(1)
        assert (st == 0).all(), "status"
        if call:
            for i in (0, 1, 12345, n - 1):
                want = b"instance output line %d%d\n" % ((i // 10) % 10, i % 10)
                assert ctx.wasi_output(i, 1) == want, (i, ctx.wasi_output(i, 1))
        return best
    finally:
        ctx.close()


def main():
    n = 65536
    out = {"what": "one host-call service round: 65,536 lanes each calling WASI fd_write once "
                   "(24 bytes to stdout), BatchRun wall time, best of 3"}
    for threads in (1, 0):
        t_call, t_none = timed(1, n, threads), timed(0, n, threads)
        key = "threads_default" if threads == 0 else "threads_1"
        out[key] = {"with_call_s": t_call, "without_call_s": t_none,
                    "round_s": t_call - t_none, "round_per_lane_us": (t_call - t_none) / n * 1e6}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
