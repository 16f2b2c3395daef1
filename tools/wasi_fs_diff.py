"""Debug aid (GPU box): run tests/test_wasi_fs.py's module on the oracle and on the GPU and
print, per mismatching lane, the first memory words that differ (offset, oracle, GPU) and
the lstat of the tree's entries before and after."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle_py as O  # noqa: E402
import test_wasi_fs as T  # noqa: E402
from wasmedge_amd import batch  # noqa: E402


def tree():
    import pathlib
    d = pathlib.Path(tempfile.mkdtemp())
    (d / "hi.txt").write_bytes(b"hello, batched wasi\n")
    (d / "sub").mkdir()
    (d / "sub" / "inner.txt").write_bytes(b"inner")
    os.symlink("hi.txt", d / "link")
    os.symlink("sub", d / "dlink")
    if os.environ.get("PIN"):   # (the test fixture's pinned times)
        now = time.time()
        for p in (d / "hi.txt", d / "sub" / "inner.txt"):
            os.utime(p, (now + 3600, now))
        os.utime(d / "sub", (now + 3600, now))
    return str(d)


def lst(d):
    return {n: (lambda s: (s.st_atime_ns, s.st_mtime_ns, s.st_ctime_ns))(os.lstat(os.path.join(d, n)))
            for n in ("hi.txt", "sub", "link", "dlink")}


d = tree()
print("fs", os.popen("stat -f -c %T " + d).read().strip(), os.popen("findmnt -T " + d + " -o OPTIONS -n").read().strip())
print("before", lst(d))
rows = [[s] for s in range(5)] * int(os.environ.get("REP", "3"))
O.set_wasi(True, ["fs.wasm"], [], preopens=[".:" + d], deterministic=(T.SEED, T.CLOCK))
m = O.Module(T.FS)
om = []
for i, r in enumerate(rows):
    inst = O.Instance(m)
    inst.set_lane(i)
    res = inst.invoke("run", r)
    om.append((res, inst.memory(0, 65536)))
print("after oracle", lst(d))
ctx = batch.BatchContext(T.FS, len(rows), device=0, host_threads=int(os.environ.get("HT", "0")))
ctx.init_wasi(["fs.wasm"], [], preopens=[".:" + d])
ctx.wasi_deterministic(T.SEED, T.CLOCK)
rets, st, cnt = ctx.execute("run", batch.make_values(rows, [batch.I32]), 1)
print("after gpu", lst(d))
for i in range(len(rows)):
    g = ctx.memory(i, 0, 65536)
    o = om[i][1]
    if g != o:
        diffs = [k for k in range(0, 65536, 4) if g[k:k + 4] != o[k:k + 4]]
        print("lane", i, "scenario", rows[i][0], "words", [(k, o[k:k + 4].hex(), g[k:k + 4].hex()) for k in diffs[:12]])
print("status", list(st), "counts", [int(c) for c in cnt][:5], [r[0][2] for r in om][:5])
