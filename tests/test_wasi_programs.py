"""The reference's own WASI command program on the yield path (VERDICT r5
"missing #1").

tools/wasmedge/examples/hello.wasm is the compiled Rust command the reference's README runs
as `wasmedge hello.wasm 1 2 3` (tools/wasmedge/examples/README.md:5-15). At startup Rust's
std (wasi-libc) walks the preopened directories from fd 3 with fd_prestat_get /
fd_prestat_dir_name until one answers BADF (lib/host/wasi/wasifunc.cpp:724-766,
include/host/wasi/environ.h:385-420), reads its command line with args_sizes_get /
args_get, and prints through fd_write.

Known answer: the README's lines "1", "2", "3" for the arguments. Its first line reads
"hello.wasm", but the module's only greeting is the literal "hello\\n" in its data section
(byte 74001 of the file) and main() skips argv[0] -- the program prints "hello", whatever
its argv[0]; the README's first line is not what this binary prints, and the tests pin the
bytes the module can produce. Every other lane is checked against the oracle's
restatement: status, instruction count, memory hash, stdout/stderr and exit code, with a
command line of its own per lane (WasmEdge_BatchWASISetInstanceArgs: the reference builds
one Environ per VM)."""
import random

import pytest

import oracle_py as O
from conftest import golden
from helpers import compare, emu_run, emu_set_wasi, emu_wasi_output
from wasmedge_amd.wat import assemble

I32 = 0x7F
README_ARGS = ["hello.wasm", "1", "2", "3"]
README_OUT = b"hello\n1\n2\n3\n"

# fd_prestat_get / fd_prestat_dir_name on every kind of fd, the name copy truncated to
# the buffer, and out-of-bounds pointers; memory around the 8-byte prestat is pre-filled
# so that the untouched padding bytes show in the memory hash
PRESTAT = assemble(r"""
(module
  (import "wasi_snapshot_preview1" "fd_prestat_get" (func $get (param i32 i32) (result i32)))
  (import "wasi_snapshot_preview1" "fd_prestat_dir_name" (func $name (param i32 i32 i32) (result i32)))
  (memory 1)
  (data (i32.const 256) "\ff\ff\ff\ff\ff\ff\ff\ff\ff\ff\ff\ff\ff\ff\ff\ff")
  (data (i32.const 512) "################################")
  (func (export "run") (param $fd i32) (param $len i32) (param $where i32) (result i32)
    (local $p i32) (local $q i32)
    (local.set $p (select (i32.const 65532) (i32.const 256) (i32.eq (local.get $where) (i32.const 1))))
    (local.set $q (select (i32.const 65530) (i32.const 512) (i32.eq (local.get $where) (i32.const 2))))
    (i32.add
      (i32.mul (call $get (local.get $fd) (local.get $p)) (i32.const 100000))
      (i32.add (i32.mul (call $name (local.get $fd) (local.get $q) (local.get $len)) (i32.const 1000))
               (i32.load8_u (i32.const 512))))))
""")
PREOPENS = [".:.", "/data/../srv/./www:/tmp", "//x/y/"]
PRESTAT_ROWS = [[fd, ln, w] for fd in (-1, 0, 1, 2, 3, 4, 5, 6, 99) for ln in (0, 1, 3, 40)
                for w in (0, 1, 2)]


def _oracle(wasm, rows, func, args_per_row=None, preopens=(), shared=README_ARGS):
    O.set_wasi(True, shared, ["HOME=/"], preopens=preopens)
    try:
        m = O.Module(wasm)
        out = []
        for i, r in enumerate(rows):
            inst = O.Instance(m)
            if args_per_row is not None and args_per_row[i] is not None:
                inst.set_args(args_per_row[i])
            res = inst.invoke(func, r)
            out.append((res, inst.wasi_output(1), inst.wasi_output(2), inst.wasi_exit_code()))
        return out
    finally:
        O.set_wasi(False)


def _lane_args(n, seed=5):
    """Lane i's command line: every fourth lane the README's, the rest random (empty
    arguments, long ones, none at all); lanes 3 mod 8 keep the shared args."""
    rng = random.Random(seed)
    out = []
    for i in range(n):
        if i % 4 == 0:
            out.append(list(README_ARGS))
        elif i % 8 == 3:
            out.append(None)
        else:
            k = rng.randrange(0, 7)
            out.append(["hello.wasm"] + ["".join(rng.choice("abcxyz0123456789-")
                                                 for _ in range(rng.randrange(0, 40)))
                                         for _ in range(k)])
    return out


def test_oracle_hello_readme():
    """The README's command line prints its arguments one per line."""
    (code, vals, cnt, _), out, err, ex = _oracle(golden("hello.wasm"), [[]], "_start")[0]
    assert code == 0 and out == README_OUT and err == b"" and ex == 0
    assert cnt > 10000


def test_oracle_prestat_known_answers():
    ref = _oracle(PRESTAT, PRESTAT_ROWS, "run", preopens=PREOPENS)
    by = {tuple(r): x[0] for r, x in zip(PRESTAT_ROWS, ref)}
    # no node -> BADF for both; stdio -> INVAL; a preopen -> SUCCESS and its name
    def val(fd, ln, w):
        v = by[(fd, ln, w)][1][0]
        return v // 100000, v % 100000 // 1000, v % 1000    # get, dir_name, first name byte
    assert val(-1, 40, 0) == (8, 8, ord("#")) and val(6, 40, 0) == (8, 8, ord("#"))
    assert val(1, 40, 0) == (28, 28, ord("#"))
    assert val(3, 40, 0) == (0, 0, ord("."))                  # "." (canonicalGuest)
    assert val(4, 40, 0) == (0, 0, ord("s"))                  # "srv/www"
    assert val(4, 0, 0) == (0, 0, ord("#"))                   # nothing copied
    # out-of-bounds prestat / name buffer -> FAULT before the fd is looked at
    assert val(-1, 40, 1)[0] == 21 and val(3, 40, 2)[1] == 21
    assert val(3, 1, 2)[1] == 0                               # 65530 + 1 in bounds


def test_emulator_prestat_matches_oracle(built):
    ref = _oracle(PRESTAT, PRESTAT_ROWS, "run", preopens=PREOPENS)
    emu_set_wasi(True, README_ARGS, ["HOME=/"], preopens=PREOPENS)
    try:
        got = emu_run(PRESTAT, "run", PRESTAT_ROWS, [I32] * 3, [I32])
    finally:
        emu_set_wasi(False)
    assert compare([r[0] for r in ref], *got, [I32]) == []


def test_emulator_hello_lane_args_match_oracle(built):
    n = 48
    largs = _lane_args(n)
    ref = _oracle(golden("hello.wasm"), [[]] * n, "_start", largs)
    emu_set_wasi(True, README_ARGS, ["HOME=/"],
                 instance_args={i: a for i, a in enumerate(largs) if a is not None})
    try:
        got = emu_run(golden("hello.wasm"), "_start", [[]] * n, [], [])
        outs = [(emu_wasi_output(i, 1), emu_wasi_output(i, 2)) for i in range(n)]
    finally:
        emu_set_wasi(False)
    assert compare([r[0] for r in ref], *got, []) == []
    assert outs == [(r[1], r[2]) for r in ref]
    assert outs[0][0] == README_OUT


def _gpu(wasm, rows, func, ptypes, nres, largs=None, preopens=(), host_threads=16, **kw):
    from wasmedge_amd import batch
    ctx = batch.BatchContext(wasm, len(rows), device=0, host_threads=host_threads, **kw)
    try:
        ctx.init_wasi(README_ARGS, ["HOME=/"], preopens=preopens)
        for i, a in enumerate(largs or []):
            if a is not None:
                ctx.set_instance_args(i, a)
        rets, st, cnt = ctx.execute(func, batch.make_values(rows, ptypes), 1)
        h = ctx.memory_hash()
        ints = batch.ret_ints(rets)
        vals = [[int(ints[i][0])] if st[i] == 0 and nres else [] for i in range(len(rows))]
        side = [(ctx.wasi_output(i, 1), ctx.wasi_output(i, 2), ctx.wasi_exit_code(i))
                for i in range(len(rows))]
        return (vals, st, cnt, h), side
    finally:
        ctx.close()


@pytest.mark.gpu
def test_gpu_prestat_matches_oracle(built):
    ref = _oracle(PRESTAT, PRESTAT_ROWS, "run", preopens=PREOPENS)
    got, side = _gpu(PRESTAT, PRESTAT_ROWS, "run", [I32] * 3, 1, preopens=PREOPENS)
    assert compare([r[0] for r in ref], *got, [I32]) == []
    assert side == [(r[1], r[2], r[3]) for r in ref]


@pytest.mark.gpu
def test_gpu_hello_4096_lanes_own_args(built):
    """hello.wasm's _start on 4,096 lanes, each with its own command line."""
    n = 4096
    largs = _lane_args(n)
    ref = _oracle(golden("hello.wasm"), [[]] * n, "_start", largs)
    got, side = _gpu(golden("hello.wasm"), [[]] * n, "_start", [], 0, largs)
    assert compare([r[0] for r in ref], *got, []) == []
    assert side == [(r[1], r[2], r[3]) for r in ref]
    assert all(side[i][0] == README_OUT for i in range(0, n, 4))
