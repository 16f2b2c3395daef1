"""QuickJS -- the largest real program the reference ships -- on the yield path (SURVEY.md §8
f1; VERDICT r5 "missing #2").

tools/wasmedge/examples/js/qjs.wasm (2.9 MB: QuickJS with a Rust WASI front end) runs as a
WASI command: `wasmedge --dir .:. qjs.wasm hello.js 1 2 3` prints `Hello 1 2 3`
(tools/wasmedge/examples/js/README.md:9-14). On the way it walks the preopens
(fd_prestat_get / _dir_name), seeds itself from clock_time_get and random_get, opens the
script under the preopened directory (path_open), stats and reads it (fd_filestat_get,
fd_read), closes it, checks stdout (fd_fdstat_get) and prints (fd_write) -- with heavy
call_indirect, malloc-driven memory.grow and ~6.5 million instructions per instance.

Scripts are the tests' own (written to a temporary directory): `hi.js` prints "Hello" and
its arguments as the README's hello.js does, so the README's answer pins its output; the
others loop for a per-lane count, throw, or name files that do not exist or lie outside the
preopen. Every lane is checked against the oracle's independent restatement of the same
WASI functions (oracle/wasi_fs.inc): status, instruction count, memory hash, stdout,
stderr and exit code. The fd numbers and random_get bytes the reference draws at random
come from the reproducible generator (WasmEdge_BatchWASISetDeterministic) on both sides; the
files' access times are set after their modification times so that reading them changes
nothing a later fd_filestat_get reports."""
import os
import random
import time

import pytest

import oracle_py as O
from conftest import golden
from helpers import compare, emu_run, emu_set_wasi, emu_wasi_output

SEED, CLOCK = 0x5EED, 1_700_000_000_000_000_000
SCRIPTS = {
    "hi.js": 'print("Hello", ...args.slice(1))\n',
    "loop.js": 'let n = +args[1], s = 0\nfor (let i = 0; i < n; i++) s += i * i % 7\nprint("sum", n, s)\n',
    "throw.js": 'function f(x) { if (x > 2) throw new Error("boom " + x); return x }\nprint(f(+args[1]))\n',
}


@pytest.fixture(scope="module")
def jsdir(tmp_path_factory):
    d = tmp_path_factory.mktemp("js")
    now = time.time()
    for name, text in SCRIPTS.items():
        p = d / name
        p.write_text(text)
        os.utime(p, (now + 3600, now))   # atime after mtime: reading it changes no stat
    return str(d)


def lane_args(n, seed=11):
    """Lane i's command line: the README's hello (every 8th lane), loops of per-lane
    length, throws, missing / out-of-preopen scripts and a missing argument."""
    rng = random.Random(seed)
    out = []
    for i in range(n):
        k = i % 8
        if k == 0:
            out.append(["qjs.wasm", "hi.js", "1", "2", "3"])
        elif k in (1, 2, 3):
            out.append(["qjs.wasm", "loop.js", str(rng.randrange(0, 600))])
        elif k == 4:
            out.append(["qjs.wasm", "throw.js", str(rng.randrange(0, 6))])
        elif k == 5:
            out.append(["qjs.wasm", "hi.js"] + [str(rng.randrange(1000)) for _ in range(rng.randrange(0, 5))])
        elif k == 6:
            out.append(["qjs.wasm", rng.choice(["missing.js", "../hi.js", "/hi.js", "./hi.js"])])
        else:
            out.append(["qjs.wasm"])
    return out


def oracle_rows(args, jsdir, lanes=None):
    """The oracle's rows for these command lines; lanes: each one's instance id (its WASI
    generator key; default 0, 1, ...)."""
    O.set_lazy_imports(True)
    O.set_wasi(True, ["qjs.wasm"], ["HOME=/"], preopens=[".:" + jsdir], deterministic=(SEED, CLOCK))
    try:
        m = O.Module(golden("qjs.wasm"))
        rows = []
        for i, a in enumerate(args):
            inst = O.Instance(m)
            inst.set_lane(lanes[i] if lanes is not None else i)
            inst.set_args(a)
            res = inst.invoke("_start", [])
            rows.append((res, inst.wasi_output(1), inst.wasi_output(2), inst.wasi_exit_code()))
        return rows
    finally:
        O.set_wasi(False)
        O.set_lazy_imports(False)


def test_oracle_readme_hello(jsdir):
    """js/README.md:9-14: Hello 1 2 3"""
    (code, _, cnt, _), out, err, ex = oracle_rows([["qjs.wasm", "hi.js", "1", "2", "3"]], jsdir)[0]
    assert code == 0 and out == b"Hello 1 2 3\n" and err == b"" and ex == 0 and cnt > 5_000_000


def test_oracle_error_paths(jsdir):
    rows = oracle_rows([["qjs.wasm", "missing.js"], ["qjs.wasm", "../hi.js"],
                        ["qjs.wasm", "throw.js", "5"], ["qjs.wasm"]], jsdir)
    assert rows[0][2] == b"No such file or directory (os error 44)\n"        # NOENT
    assert rows[1][2] == b"Capabilities insufficient (os error 76)\n"        # ".." past the preopen
    assert rows[2][2].startswith(b"Error: boom 5\n")
    assert rows[3][0][0] == O.TERMINATED and rows[3][3] == 2                 # proc_exit(2)


def test_emulator_matches_oracle(built, jsdir):
    args = lane_args(16)
    ref = oracle_rows(args, jsdir)
    emu_set_wasi(True, ["qjs.wasm"], ["HOME=/"], preopens=[".:" + jsdir],
                 instance_args=dict(enumerate(args)), deterministic=(SEED, CLOCK))
    try:
        got = emu_run(golden("qjs.wasm"), "_start", [[]] * len(args), [], [])
        side = [(emu_wasi_output(i, 1), emu_wasi_output(i, 2)) for i in range(len(args))]
    finally:
        emu_set_wasi(False)
    assert compare([r[0] for r in ref], *got, []) == []
    assert side == [(r[1], r[2]) for r in ref]
    assert side[0][0] == b"Hello 1 2 3\n"


@pytest.mark.gpu
def test_gpu_quickjs_512_lanes(built, jsdir, monkeypatch):
    """512 instances of QuickJS (8 waves), each with its own command line, on the threaded
    core (WB_JIT=0: the 64,000 compiled runs of this module take about a minute of hiprtc
    at BatchCreate; tools/qjs_gpu.py runs them at scale), host calls on 16 threads."""
    from wasmedge_amd import batch
    monkeypatch.setenv("WB_JIT", "0")
    args = lane_args(512)
    ref = oracle_rows(args, jsdir)
    ctx = batch.BatchContext(golden("qjs.wasm"), len(args), device=0, host_threads=16)
    try:
        ctx.init_wasi(["qjs.wasm"], ["HOME=/"], preopens=[".:" + jsdir])
        ctx.wasi_deterministic(SEED, CLOCK)
        for i, a in enumerate(args):
            ctx.set_instance_args(i, a)
        _, st, cnt = ctx.execute("_start", batch.make_values([[]] * len(args), []), 0)
        h = ctx.memory_hash()
        side = [(ctx.wasi_output(i, 1), ctx.wasi_output(i, 2), ctx.wasi_exit_code(i))
                for i in range(len(args))]
    finally:
        ctx.close()
    assert compare([r[0] for r in ref], [[]] * len(args), st, cnt, h, []) == []
    assert side == [(r[1], r[2], r[3]) for r in ref]
    assert all(side[i][0] == b"Hello 1 2 3\n" for i in range(0, len(args), 8))
