"""QuickJS (the reference's qjs.wasm) on the GPU at scale, with the compiled runs on or off
(WB_JIT), every lane checked against the oracle on a sample: prints create time, run time,
instructions and the aggregate rate. usage: python tools/qjs_gpu.py N [sample]"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import test_quickjs as Q  # noqa: E402
from helpers import compare  # noqa: E402
from wasmedge_amd import batch  # noqa: E402


def main():
    n = int(sys.argv[1])
    sample = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    d = tempfile.mkdtemp()
    now = time.time()
    for name, text in Q.SCRIPTS.items():
        p = os.path.join(d, name)
        open(p, "w").write(text)
        os.utime(p, (now + 3600, now))
    args = Q.lane_args(n)
    wasm = open(os.path.join(ROOT, "tests", "golden", "qjs.wasm"), "rb").read()
    t = time.perf_counter()
    ctx = batch.BatchContext(wasm, n, device=0, host_threads=16)
    t_create = time.perf_counter() - t
    ctx.init_wasi(["qjs.wasm"], ["HOME=/"], preopens=[".:" + d])
    ctx.wasi_deterministic(Q.SEED, Q.CLOCK)
    for i, a in enumerate(args):
        ctx.set_instance_args(i, a)
    t = time.perf_counter()
    _, st, cnt = ctx.execute("_start", batch.make_values([[]] * n, []), 0)
    t_run = time.perf_counter() - t
    h = ctx.memory_hash()
    idx = list(range(0, n, max(1, n // sample)))
    ref = Q.oracle_rows([args[i] for i in idx], d, lanes=idx)
    bad = compare([r[0] for r in ref], [[]] * len(idx), st[idx], cnt[idx], h[idx], [])
    outs = [(ctx.wasi_output(i, 1), ctx.wasi_output(i, 2)) for i in idx]
    print({"n": n, "jit": os.environ.get("WB_JIT", "1"), "compiled_runs": ctx.compiled_runs(),
           "engine": ctx.engine(), "create_s": round(t_create, 2), "run_s": round(t_run, 3),
           "instrs": int(cnt.sum()), "instr_per_s": float(cnt.sum()) / t_run,
           "sample": len(idx), "mismatches": len(bad), "first": bad[:3],
           "stdout_ok": sum(o[0] == r[1] and o[1] == r[2] for o, r in zip(outs, ref))})
    ctx.close()


if __name__ == "__main__":
    main()
