"""The WASI file, clock and random subset, function by function.

One module drives path_open, fd_read, fd_seek, fd_tell, fd_close, fd_fdstat_get,
fd_fdstat_set_flags, fd_filestat_get, path_filestat_get, fd_prestat_get, clock_time_get,
clock_res_get and random_get through their error paths against a preopened directory
(regular file, subdirectory, symbolic links). Each scenario leaves its errnos and every byte
the functions wrote in linear memory; the library's restatement (wasmedge_amd/csrc/
wasi_impl.h: the emulator on the CPU, the batched path on the GPU) is compared with the
oracle's (oracle/wasi_fs.inc) -- status, count, memory hash -- on every scenario. What the
reference does per case is cited in both restatements; the preopen is a read-only mount
here (ROFS for opens that would write), and fd numbers / random bytes / clocks come from
the reproducible generator (WasmEdge_BatchWASISetDeterministic) on both sides. Parity with
the reference beyond the restatements is unpinned: no reference fixture exercises these."""
import os
import time

import pytest

import oracle_py as O
from helpers import compare, emu_run, emu_set_wasi
from wasmedge_amd.wat import assemble

I32 = 0x7F
SEED, CLOCK = 99, 1_650_000_000_000_000_000
W = "wasi_snapshot_preview1"

FS = assemble(r"""
(module
  (import "%(W)s" "path_open" (func $open (param i32 i32 i32 i32 i32 i64 i64 i32 i32) (result i32)))
  (import "%(W)s" "fd_read" (func $read (param i32 i32 i32 i32) (result i32)))
  (import "%(W)s" "fd_write" (func $write (param i32 i32 i32 i32) (result i32)))
  (import "%(W)s" "fd_seek" (func $seek (param i32 i64 i32 i32) (result i32)))
  (import "%(W)s" "fd_tell" (func $tell (param i32 i32) (result i32)))
  (import "%(W)s" "fd_close" (func $close (param i32) (result i32)))
  (import "%(W)s" "fd_fdstat_get" (func $fdstat (param i32 i32) (result i32)))
  (import "%(W)s" "fd_fdstat_set_flags" (func $setflags (param i32 i32) (result i32)))
  (import "%(W)s" "fd_filestat_get" (func $filestat (param i32 i32) (result i32)))
  (import "%(W)s" "path_filestat_get" (func $pstat (param i32 i32 i32 i32 i32) (result i32)))
  (import "%(W)s" "fd_prestat_get" (func $prestat (param i32 i32) (result i32)))
  (import "%(W)s" "clock_time_get" (func $clock (param i32 i64 i32) (result i32)))
  (import "%(W)s" "clock_res_get" (func $res (param i32 i32) (result i32)))
  (import "%(W)s" "random_get" (func $rand (param i32 i32) (result i32)))
  (memory 1)
  ;; path strings at 100 + 16 * k: hi.txt sub link dlink nope/x hi.txt/x ../x /hi.txt . sub/../hi.txt
  (data (i32.const 100) "hi.txt")
  (data (i32.const 116) "sub")
  (data (i32.const 132) "link")
  (data (i32.const 148) "dlink")
  (data (i32.const 164) "nope/x")
  (data (i32.const 180) "hi.txt/x")
  (data (i32.const 196) "../x")
  (data (i32.const 212) "/hi.txt")
  (data (i32.const 228) ".")
  (data (i32.const 244) "sub/../hi.txt")
  (data (i32.const 260) "../hi.txt")
  (global $o (mut i32) (i32.const 1024))   ;; the next result slot
  (func $put (param $v i32) (i32.store (global.get $o) (local.get $v))
    (global.set $o (i32.add (global.get $o) (i32.const 4))))
  ;; path k (its length from the table at 300), rights and flags as given; the fd -> 900
  (func $op (param $dir i32) (param $look i32) (param $k i32) (param $of i32) (param $rb i64) (result i32)
    (call $open (local.get $dir) (local.get $look) (i32.add (i32.const 100) (i32.mul (local.get $k) (i32.const 16)))
      (i32.load8_u (i32.add (i32.const 300) (local.get $k))) (local.get $of) (local.get $rb) (local.get $rb)
      (i32.const 0) (i32.const 900)))
  (data (i32.const 300) "\06\03\04\05\06\08\04\07\01\0d\09")
  ;; iovec at 880: 64 bytes at 2048
  (data (i32.const 880) "\00\08\00\00\40\00\00\00")
  (func (export "run") (param $s i32) (result i32)
    (local $fd i32) (local $sub i32)
    (if (i32.eq (local.get $s) (i32.const 0)) (then   ;; read, tell, seek, stat, close
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 0) (i64.const 0x2000a6)))
      (local.set $fd (i32.load (i32.const 900)))
      (i32.store (i32.const 884) (i32.const 5))
      (call $put (call $read (local.get $fd) (i32.const 880) (i32.const 1) (i32.const 904)))
      (call $put (call $tell (local.get $fd) (i32.const 912)))
      (call $put (call $seek (local.get $fd) (i64.const -2) (i32.const 1) (i32.const 920)))
      (i32.store (i32.const 880) (i32.const 2100))
      (i32.store (i32.const 884) (i32.const 100))
      (call $put (call $read (local.get $fd) (i32.const 880) (i32.const 1) (i32.const 928)))
      (call $put (call $seek (local.get $fd) (i64.const 3) (i32.const 2) (i32.const 936)))
      (call $put (call $seek (local.get $fd) (i64.const -100) (i32.const 2) (i32.const 944)))
      (call $put (call $seek (local.get $fd) (i64.const 0) (i32.const 3) (i32.const 944)))
      (call $put (call $seek (local.get $fd) (i64.const 1) (i32.const 0x100) (i32.const 944)))
      (call $put (call $filestat (local.get $fd) (i32.const 3000)))
      (call $put (call $fdstat (local.get $fd) (i32.const 3100)))
      (call $put (call $write (local.get $fd) (i32.const 880) (i32.const 1) (i32.const 950)))
      (call $put (call $setflags (local.get $fd) (i32.const 0)))
      (call $put (call $close (local.get $fd)))
      (call $put (call $close (local.get $fd)))
      (call $put (call $read (local.get $fd) (i32.const 880) (i32.const 1) (i32.const 904)))))
    (if (i32.eq (local.get $s) (i32.const 1)) (then   ;; opens that write, create, truncate
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 1) (i64.const 2)))    ;; CREAT existing
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 4) (i32.const 1) (i64.const 2)))    ;; CREAT new (nope/x)
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 1) (i32.const 1) (i64.const 2)))    ;; CREAT on a dir
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 5) (i64.const 2)))    ;; CREAT|EXCL
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 8) (i64.const 2)))    ;; TRUNC
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 0) (i64.const 0x40)))  ;; FD_WRITE
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 1) (i32.const 0) (i64.const 0x40)))  ;; write a dir
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 2) (i64.const 2)))))  ;; DIRECTORY on a file
    (if (i32.eq (local.get $s) (i32.const 2)) (then   ;; resolution
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 1) (i32.const 2) (i64.const 0x4002)))
      (local.set $sub (i32.load (i32.const 900)))
      (i32.store (i32.const 884) (i32.const 8))
      (call $put (call $read (local.get $sub) (i32.const 880) (i32.const 1) (i32.const 904)))        ;; ISDIR
      (call $put (call $op (local.get $sub) (i32.const 0) (i32.const 10) (i32.const 0) (i64.const 2))) ;; ../hi.txt
      (call $put (call $op (local.get $sub) (i32.const 0) (i32.const 6) (i32.const 0) (i64.const 2)))  ;; ../x
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 6) (i32.const 0) (i64.const 2)))      ;; ../x at the top
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 4) (i32.const 0) (i64.const 2)))      ;; nope/x
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 5) (i32.const 0) (i64.const 2)))      ;; hi.txt/x
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 2) (i32.const 0) (i64.const 2)))      ;; link, no follow
      (call $put (call $op (i32.const 3) (i32.const 1) (i32.const 2) (i32.const 0) (i64.const 2)))      ;; link, follow
      (call $put (call $op (i32.const 3) (i32.const 1) (i32.const 3) (i32.const 2) (i64.const 2)))      ;; dlink -> sub
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 7) (i32.const 0) (i64.const 2)))      ;; /hi.txt
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 8) (i32.const 2) (i64.const 0x4002)))   ;; .
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 9) (i32.const 0) (i64.const 2)))      ;; sub/../hi.txt
      (call $put (call $op (i32.const 0) (i32.const 0) (i32.const 0) (i32.const 0) (i64.const 2)))      ;; from stdin
      (call $put (call $op (i32.const 77) (i32.const 0) (i32.const 0) (i32.const 0) (i64.const 2)))     ;; no such fd
      (call $put (call $open (i32.const 3) (i32.const 0) (i32.const 100) (i32.const 0) (i32.const 0)
                   (i64.const 2) (i64.const 2) (i32.const 0) (i32.const 900)))                         ;; empty path
      (call $put (call $pstat (i32.const 3) (i32.const 0) (i32.const 132) (i32.const 4) (i32.const 3200)))
      (call $put (call $pstat (i32.const 3) (i32.const 1) (i32.const 132) (i32.const 4) (i32.const 3300)))
      (call $put (call $pstat (i32.const 3) (i32.const 0) (i32.const 116) (i32.const 3) (i32.const 3400)))
      (call $put (call $pstat (i32.const 3) (i32.const 0) (i32.const 164) (i32.const 6) (i32.const 3500)))
      (call $put (call $pstat (i32.const 3) (i32.const 2) (i32.const 100) (i32.const 6) (i32.const 3500)))))
    (if (i32.eq (local.get $s) (i32.const 3)) (then   ;; flags, pointers, stdio, preopen
      (call $put (call $op (i32.const 3) (i32.const 2) (i32.const 0) (i32.const 0) (i64.const 2)))      ;; dirflags
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 0x10) (i64.const 2)))   ;; oflags
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 0x10000) (i64.const 2))) ;; u16 cast
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 0) (i64.const 0x1000000000)))  ;; rights
      (call $put (call $open (i32.const 3) (i32.const 0) (i32.const 65534) (i32.const 6) (i32.const 0)
                   (i64.const 2) (i64.const 2) (i32.const 0) (i32.const 900)))                          ;; path OOB
      (call $put (call $open (i32.const 3) (i32.const 0) (i32.const 100) (i32.const 6) (i32.const 0)
                   (i64.const 2) (i64.const 2) (i32.const 0) (i32.const 65534)))                        ;; fd OOB
      (call $put (call $open (i32.const 3) (i32.const 0) (i32.const 100) (i32.const 6) (i32.const 0)
                   (i64.const 2) (i64.const 2) (i32.const 0x20) (i32.const 900)))                       ;; fdflags
      (call $put (call $seek (i32.const 1) (i64.const 0) (i32.const 0) (i32.const 960)))
      (call $put (call $tell (i32.const 0) (i32.const 960)))
      (call $put (call $fdstat (i32.const 1) (i32.const 3600)))
      (call $put (call $fdstat (i32.const 3) (i32.const 3700)))
      (call $put (call $fdstat (i32.const 99) (i32.const 3800)))
      (call $put (call $fdstat (i32.const 1) (i32.const 65530)))
      (call $put (call $filestat (i32.const 1) (i32.const 3900)))
      (call $put (call $filestat (i32.const 3) (i32.const 4000)))
      (call $put (call $setflags (i32.const 1) (i32.const 0)))
      (call $put (call $setflags (i32.const 3) (i32.const 1)))
      (call $put (call $setflags (i32.const 3) (i32.const 0x40)))
      (i32.store (i32.const 884) (i32.const 8))
      (call $put (call $read (i32.const 0) (i32.const 880) (i32.const 1) (i32.const 904)))      ;; stdin: EOF
      (call $put (call $close (i32.const 3)))                                                   ;; preopen
      (call $put (call $close (i32.const 2)))
      (call $put (call $write (i32.const 2) (i32.const 880) (i32.const 1) (i32.const 904)))     ;; closed
      (call $put (call $prestat (i32.const 2) (i32.const 970)))))
    (if (i32.eq (local.get $s) (i32.const 4)) (then   ;; clocks and random bytes
      (call $put (call $clock (i32.const 0) (i64.const 1) (i32.const 4096)))
      (call $put (call $clock (i32.const 1) (i64.const 1) (i32.const 4104)))
      (call $put (call $clock (i32.const 4) (i64.const 1) (i32.const 4112)))
      (call $put (call $clock (i32.const 0) (i64.const 1) (i32.const 65535)))
      (call $put (call $res (i32.const 1) (i32.const 4120)))
      (call $put (call $rand (i32.const 4200) (i32.const 7)))
      (call $put (call $rand (i32.const 4210) (i32.const 0)))
      (call $put (call $rand (i32.const 65533) (i32.const 4)))
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 0) (i64.const 2)))   ;; fd numbers
      (call $put (i32.load (i32.const 900)))
      (call $put (call $op (i32.const 3) (i32.const 0) (i32.const 0) (i32.const 0) (i64.const 2)))
      (call $put (i32.load (i32.const 900)))))
    (i32.load (i32.const 1024))))
""" % {"W": W})

ROWS = [[s] for s in range(5)] * 13


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    d = tmp_path_factory.mktemp("tree")
    (d / "hi.txt").write_bytes(b"hello, batched wasi\n")
    (d / "sub").mkdir()
    (d / "sub" / "inner.txt").write_bytes(b"inner")
    os.symlink("hi.txt", d / "link")
    os.symlink("sub", d / "dlink")
    # access times after the modification and change times, so that no read (relatime)
    # changes what a later stat reports -- the symbolic links too: readlink would otherwise
    # update a link's atime while it still equals its mtime, which on the coarse file clock
    # can last past the first read
    now = time.time()
    for p in (d / "hi.txt", d / "sub" / "inner.txt", d / "sub"):
        os.utime(p, (now + 3600, now))
    for p in (d / "link", d / "dlink"):
        os.utime(p, (now + 3600, now), follow_symlinks=False)
    return str(d)


def _oracle(tree, rows, mems=None):
    O.set_wasi(True, ["fs.wasm"], [], preopens=[".:" + tree], deterministic=(SEED, CLOCK))
    try:
        m = O.Module(FS)
        out = []
        for i, r in enumerate(rows):
            inst = O.Instance(m)
            inst.set_lane(i)
            out.append(inst.invoke("run", r))
            if mems is not None:
                mems.append(inst.memory(0, 8192))
        return out
    finally:
        O.set_wasi(False)


def test_oracle_fs_known_answers(tree):
    """A few answers fixed by the reference's code paths (errno values: api.hpp)."""
    O.set_wasi(True, ["fs.wasm"], [], preopens=[".:" + tree], deterministic=(SEED, CLOCK))
    try:
        m = O.Module(FS)
        inst = O.Instance(m)
        assert inst.invoke("run", [1])[0] == 0
        errs = [int.from_bytes(inst.memory(1024 + 4 * k, 4), "little") for k in range(8)]
        inst2 = O.Instance(m)
        inst2.invoke("run", [2])
        res = [int.from_bytes(inst2.memory(1024 + 4 * k, 4), "little") for k in range(22)]
    finally:
        O.set_wasi(False)
    # CREAT of an existing file opens it, CREAT under a missing dir -> NOENT, CREAT of a
    # dir -> ISDIR, CREAT|EXCL -> EXIST, TRUNC -> ROFS (read-only mount), FD_WRITE -> ROFS,
    # write access to a dir -> ISDIR, DIRECTORY on a file -> NOTDIR
    assert errs == [0, 44, 31, 20, 69, 69, 31, 54]
    assert res[1] == 31                      # fd_read on a directory: ISDIR
    assert res[2] == 0 and res[3] == 44      # ../hi.txt from sub; ../x from sub: no such file
    assert res[4] == 76                      # ../x at the preopen: past it, NOTCAPABLE
    assert res[5] == 44 and res[6] == 54     # nope/x, hi.txt/x
    assert res[7] == 32 and res[8] == 0      # a symlink: LOOP unless followed
    assert res[13] == 54 and res[14] == 8 and res[15] == 44   # stdin no dir, no fd, empty path


def test_emulator_fs_matches_oracle(built, tree):
    ref = _oracle(tree, ROWS)
    emu_set_wasi(True, ["fs.wasm"], [], preopens=[".:" + tree], deterministic=(SEED, CLOCK))
    try:
        got = emu_run(FS, "run", ROWS, [I32], [I32])
    finally:
        emu_set_wasi(False)
    assert compare(ref, *got, [I32]) == []


@pytest.mark.gpu
def test_gpu_fs_matches_oracle(built, tree):
    from wasmedge_amd import batch
    rows = ROWS * 3
    mems = []
    ref = _oracle(tree, rows, mems)
    ctx = batch.BatchContext(FS, len(rows), device=0, host_threads=8)
    try:
        ctx.init_wasi(["fs.wasm"], [], preopens=[".:" + tree])
        ctx.wasi_deterministic(SEED, CLOCK)
        rets, st, cnt = ctx.execute("run", batch.make_values(rows, [I32]), 1)
        ints = batch.ret_ints(rets)
        vals = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(rows))]
        bad = compare(ref, vals, st, cnt, ctx.memory_hash(), [I32])
        # (on a mismatch: the first lane's differing words, oracle vs GPU)
        words = []
        if bad:
            i = bad[0][0]
            g = ctx.memory(i, 0, 8192)
            words = [(k, mems[i][k:k + 4].hex(), g[k:k + 4].hex()) for k in range(0, 8192, 4)
                     if mems[i][k:k + 4] != g[k:k + 4]][:16]
        assert bad == [], (len(bad), words)
    finally:
        ctx.close()
