"""Compiled straight-line runs (wasmedge_amd/csrc/jit.cpp, DESIGN.md "Compiled runs").

The V-frame threaded core runs a straight-line stretch of instructions as machine code
compiled for the module at BatchCreate (hiprtc, gfx950). It must give exactly what the
interpreter gives, so the same modules run against the oracle with the compiler on and
off (WB_JIT=0), bit for bit: return values, status, instruction counts, memory hash.

Random modules (seeded, generated below) cover every instruction the compiler knows:
i32/i64 arithmetic, shifts and rotates by registers and constants, compares, selects,
extensions, the fused ARX forms with aliased cells, and loads/stores of every width at
in-bounds, misaligned (the run leaves; the C++ step executes the access) and
out-of-bounds (0x88 trap at the exact instruction) addresses, under both arms of a
lane-divergent branch (the core's diverged mode) and in a loop. The CPU tests assemble
every run of the BASELINE workloads and the random modules for gfx950 at every
memory granule without a GPU."""
import ctypes
import os
import random

import pytest

import oracle_py as O
from helpers import compare, gpu_run
from wasmedge_amd import workloads as W
from wasmedge_amd.wat import assemble

I32, I64 = 0x7F, 0x7E
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N32, N64 = 6, 6

I32_BIN = ["add", "sub", "mul", "and", "or", "xor", "shl", "shr_s", "shr_u", "rotl", "rotr"]
I32_CMP = ["eq", "ne", "lt_s", "lt_u", "gt_s", "gt_u", "le_s", "le_u", "ge_s", "ge_u"]
I32_UN = ["clz", "ctz", "popcnt", "extend8_s", "extend16_s", "eqz"]
I64_BIN = I32_BIN
I64_UN = ["extend8_s", "extend16_s", "extend32_s"]
LOADS32 = [("i32.load", 4), ("i32.load8_s", 1), ("i32.load8_u", 1), ("i32.load16_s", 2), ("i32.load16_u", 2)]
LOADS64 = [("i64.load", 8), ("i64.load8_s", 1), ("i64.load8_u", 1), ("i64.load16_s", 2),
           ("i64.load16_u", 2), ("i64.load32_s", 4), ("i64.load32_u", 4)]
STORES32 = [("i32.store", 4), ("i32.store8", 1), ("i32.store16", 2)]
STORES64 = [("i64.store", 8), ("i64.store8", 1), ("i64.store16", 2), ("i64.store32", 4)]
CONSTS = [0, 1, 3, 7, 16, 31, 32, 33, 63, 64, 65, 255, -1, -16, -17, 0x7FFFFFFF, -0x80000000, 0x12345678]


def _g32(r):
    return "(local.get $a%d)" % r.randrange(N32)


def _g64(r):
    return "(local.get $b%d)" % r.randrange(N64)


def _c32(r):
    return "(i32.const %d)" % r.choice(CONSTS)


def _c64(r):
    return "(i64.const %d)" % r.choice(CONSTS + [0x123456789ABCDEF, -0x8000000000000000])


def _addr(r, n):
    """an address expression: mostly in bounds and aligned, sometimes misaligned (the run
    leaves) or past the one-page memory (0x88)"""
    k = r.random()
    if k < 0.85:
        return "(i32.and %s (i32.const %d))" % (_g32(r), 0x7FF0 & ~(max(n, 4) - 1)), \
            r.choice([0, 0, 4, 8, 12, 60, 256])
    if k < 0.99:
        return "(i32.and %s (i32.const %d))" % (_g32(r), 0xFFFF), r.choice([0, 1, 3])
    return "(i32.and %s (i32.const %d))" % (_g32(r), 0x1FFFC), 0


def _stmt(r, calls=True):
    k = r.randrange(16 if calls else 15)
    if k == 15:   # a call: the callee's locals start at zero (some read before written)
        return "(local.set $b%d (call $h (local.get $a%d) (local.get $b%d)))" % (
            r.randrange(N64), r.randrange(N32), r.randrange(N64))
    d32, d64 = "$a%d" % r.randrange(N32), "$b%d" % r.randrange(N64)
    if k == 0:
        return "(local.set %s (i32.%s %s %s))" % (d32, r.choice(I32_BIN), _g32(r), _g32(r))
    if k == 1:
        return "(local.set %s (i32.%s %s %s))" % (d32, r.choice(I32_BIN), _g32(r), _c32(r))
    if k == 2:
        return "(local.set %s (i32.%s %s %s))" % (d32, r.choice(I32_CMP), _g32(r), r.choice([_g32(r), _c32(r)]))
    if k == 3:
        u = r.choice(I32_UN)
        return "(local.set %s (i32.%s %s))" % (d32, u, _g32(r))
    if k == 4:
        return "(local.set %s (i64.%s %s %s))" % (d64, r.choice(I64_BIN), _g64(r), r.choice([_g64(r), _c64(r)]))
    if k == 5:
        return "(local.set %s (i64.%s %s %s))" % (d32, r.choice(I32_CMP), _g64(r), r.choice([_g64(r), _c64(r)]))
    if k == 6:
        return r.choice(["(local.set %s (i64.%s %s))" % (d64, r.choice(I64_UN), _g64(r)),
                         "(local.set %s (i64.extend_i32_%s %s))" % (d64, r.choice("su"), _g32(r)),
                         "(local.set %s (i32.wrap_i64 %s))" % (d32, _g64(r)),
                         "(local.set %s (i64.eqz %s))" % (d32, _g64(r))])
    if k == 7:
        return r.choice(["(local.set %s (select %s %s %s))" % (d32, _g32(r), _g32(r), _g32(r)),
                         "(local.set %s (select %s %s %s))" % (d64, _g64(r), _g64(r), _g32(r))])
    if k in (8, 9):   # BLAKE3-style quarter round on random (possibly aliased) locals
        a, b, c, d = ("$a%d" % r.randrange(N32) for _ in range(4))
        m = _g32(r)
        rot = r.choice([16, 12, 8, 7, 1, 31])
        return ("(local.set %s (i32.add (i32.add (local.get %s) (local.get %s)) %s))"
                "(local.set %s (i32.rotr (i32.xor (local.get %s) (local.get %s)) (i32.const %d)))"
                "(local.set %s (i32.add (local.get %s) (local.get %s)))"
                "(local.set %s (i32.rotr (i32.xor (local.get %s) (local.get %s)) (i32.const %d)))"
                % (a, a, b, m, d, d, a, rot, c, c, d, b, b, c, r.choice([12, 7, 9])))
    if k == 10:
        ins, n = r.choice(LOADS32)
        ad, off = _addr(r, n)
        return "(local.set %s (%s offset=%d %s))" % (d32, ins, off, ad)
    if k == 11:
        ins, n = r.choice(LOADS64)
        ad, off = _addr(r, n)
        return "(local.set %s (%s offset=%d %s))" % (d64, ins, off, ad)
    if k == 12:
        ins, n = r.choice(STORES32)
        ad, off = _addr(r, n)
        return "(%s offset=%d %s %s)" % (ins, off, ad, _g32(r))
    if k == 13:
        ins, n = r.choice(STORES64)
        ad, off = _addr(r, n)
        return "(%s offset=%d %s %s)" % (ins, off, ad, _g64(r))
    if r.random() < 0.3:
        # a load-scan loop (jit.cpp scan loops: 8 iterations per trip): up or down by a
        # word from a per-lane start, on while the loaded word compares true; zero words
        # stop the `gt_u` form at once, the `lt_u` form runs through them to the end of
        # memory (the unrolled window fails its bounds check first, then the plain run
        # traps with 0x88 at the exact instruction)
        x, y = "$a%d" % r.randrange(N32), "$a%d" % r.randrange(N32)
        if x == y:
            y = "$a%d" % ((int(x[2:]) + 1) % N32)
        cmp = r.choice(["gt_u", "lt_u"])
        lim = "(local.get %s)" % y if cmp == "gt_u" else "(i32.and (local.get %s) (i32.const 7))" % y
        lab = r.randrange(1 << 30)
        return ("(local.set %s (i32.and (local.get %s) (i32.const 0xFFFC)))"
                "(loop $s%d (local.set %s (i32.%s (local.get %s) (i32.const 4)))"
                "(br_if $s%d (i32.%s (i32.load offset=%d (local.get %s)) %s)))"
                % (x, x, lab, x, r.choice(["add", "sub"]), x, lab, cmp, r.choice([0, 4, 256]), x, lim))
    return "(local.set %s (i32.%s %s %s))" % (d32, r.choice(["add", "sub", "xor"]), _g32(r), _c32(r))


def random_module(seed, n=40):
    r = random.Random(seed)
    body = lambda: "\n    ".join(_stmt(r) for _ in range(n))
    locs = " ".join("(local $a%d i32)" % i for i in range(1, N32)) + " " + \
        " ".join("(local $b%d i64)" % i for i in range(N64))
    init = "\n    ".join(["(local.set $a%d (i32.mul (local.get $a0) (i32.const %d)))" % (i, 2654435761 * (i + 1) & 0x7FFFFFFF)
                          for i in range(1, N32)] +
                         ["(local.set $b%d (i64.mul (i64.extend_i32_u (local.get $a%d)) (i64.const %d)))" %
                          (i, i % N32, 0x9E3779B97F4A7C15 * (i + 3) & 0x7FFFFFFFFFFFFFFF) for i in range(N64)])
    fold = " ".join(["(i64.xor"] * (N32 + N64 - 1))
    parts = ["(local.get $b0)"] + ["(local.get $b%d))" % i for i in range(1, N64)] + \
        ["(i64.extend_i32_u (local.get $a%d)))" % i for i in range(N32)]
    # the callee: params $a0 $b0, locals $a1.. $b1..; its straight-line body reads some
    # locals before writing them (zero) and writes others first
    hbody = "\n    ".join(_stmt(r, calls=False) for _ in range(12))
    hlocs = " ".join("(local $a%d i32)" % i for i in range(1, N32)) + " " + \
        " ".join("(local $b%d i64)" % i for i in range(1, N64))
    hfold = "(i64.xor (local.get $b1) (i64.xor (local.get $b0) (i64.extend_i32_u (i32.add (local.get $a0) (local.get $a1)))))"
    return assemble("""
(module
  (memory 1)
  (func $h (param $a0 i32) (param $b0 i64) (result i64)
    %s
    (local.set $a2 (i32.const 5)) (local.set $b2 (i64.const 7))
    %s
    %s)
  (func (export "run") (param $a0 i32) (result i64)
    %s (local $it i32)
    %s
    %s
    (if (i32.and (local.get $a0) (i32.const 1))
      (then %s)
      (else %s))
    (loop $l
      %s
      (local.set $it (i32.add (local.get $it) (i32.const 1)))
      (br_if $l (i32.lt_u (local.get $it) (i32.const 2))))
    %s
    %s %s))
""" % (hlocs, hbody, hfold, locs, init, body(), body(), body(), body(), body(), fold, " ".join(parts)))


SEEDS = list(range(12))
ROWS = [[(i * 2654435761 + 12345) & 0xFFFFFFFF] for i in range(256)]


def _check_lib():
    L = ctypes.CDLL(os.path.join(ROOT, "wasmedge_amd", "libwasmedge_batch.so"))
    L.wb_jit_check.restype = ctypes.c_int
    L.wb_jit_check.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                               ctypes.POINTER(ctypes.c_uint32), ctypes.c_char_p, ctypes.c_uint32]
    return L


def _jit_check(wasm, glog):
    err = ctypes.create_string_buffer(4096)
    ins = ctypes.c_uint32(0)
    n = _check_lib().wb_jit_check(wasm, len(wasm), glog, ctypes.byref(ins), err, 4096)
    assert n >= 0, err.value.decode()
    return n, ins.value


def test_random_modules_run_on_oracle():
    """the generator's modules validate and exercise every outcome: success, 0x88"""
    codes = set()
    for s in SEEDS[:4]:
        m = O.Module(random_module(s))
        codes |= {m.run("run", r)[0] for r in ROWS[:64]}
    assert 0 in codes and 0x88 in codes


@pytest.mark.parametrize("glog", [0, 2, 5])
def test_runs_assemble(built, glog):
    """every compiled run of the workloads and random modules assembles for gfx950"""
    mods = [W.blake3_wasm(), W.qsort_wasm(), W.collatz_wasm(), W.mandel_wasm()] + \
        [random_module(s) for s in SEEDS[:6]]
    got = [_jit_check(m, glog) for m in mods]
    assert got[0][0] >= 1 and got[0][1] >= 250     # C2: the whole compression is one run
    assert all(n > 0 for n, _ in got[4:])


@pytest.mark.gpu
@pytest.mark.parametrize("jit", ["1", "0", "trip"])
@pytest.mark.parametrize("granule", [4, 16, 128])
def test_gpu_random_modules(built, monkeypatch, jit, granule):
    """jit "trip": trip mode forced on (WB_TRIP=1), "1" with it off"""
    monkeypatch.setenv("WB_TRIP", "1" if jit == "trip" else "0")
    if jit == "trip":
        jit = "1"
    monkeypatch.setenv("WB_JIT", jit)
    runs = 0
    for s in SEEDS:
        wasm = random_module(s)
        ref = [O.Module(wasm).run("run", r) for r in ROWS]
        from wasmedge_amd import batch
        ctx = batch.BatchContext(wasm, len(ROWS), memory_granule=granule)
        try:
            runs += ctx.compiled_runs()
            rets, st, cnt = ctx.execute("run", batch.make_values(ROWS, [I32]), 1)
            h = ctx.memory_hash()
            ints = batch.ret_ints(rets)
            rows = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(ROWS))]
        finally:
            ctx.close()
        assert compare(ref, rows, st, cnt, h, [I64], exact=True) == [], s
    assert (runs > 0) == (jit == "1")


@pytest.mark.gpu
def test_gpu_blake3_compiled(built):
    """C2's compression as one compiled run, against the oracle"""
    wasm = W.blake3_wasm()
    rows = [[i, 20] for i in range(4096)]
    m = O.Module(wasm)
    ref = [m.run("run", r) for r in rows[:512]]
    from wasmedge_amd import batch
    ctx = batch.BatchContext(wasm, len(rows))
    try:
        assert ctx.compiled_runs() >= 1
        rets, st, cnt = ctx.execute("run", batch.make_values(rows, [I32, I32]), 1)
        h = ctx.memory_hash()
        ints = batch.ret_ints(rets)
    finally:
        ctx.close()
    got = [[int(ints[i][0])] if st[i] == 0 else [] for i in range(len(rows))]
    assert compare(ref, got[:512], st[:512], cnt[:512], h[:512], [I32], exact=True) == []


def test_large_module_assembles(built):
    """The reference's 1.7 MB Rust example compiles to ~2,000 runs spread over a code
    object far beyond s_branch's +-128 KiB: run-to-run jumps are long jumps, and the
    address table keeps the compile to a couple of seconds."""
    from conftest import golden
    n, ins = _jit_check(golden("rust_add.wasm"), 0)
    assert n > 1000 and ins > 5000


def test_trip_mode_choice(built):
    """Which modules run trip mode (jit.h trips_pay, Program::divergent_mem): C3 (addresses
    from loaded data) and C4 (a br_table state machine, no calls) do; C1 (recursion), C2
    (converged, with calls), C5 (an escape loop whose lanes leave one by one) do not."""
    L = _check_lib()
    L.wb_trip_choice.restype = ctypes.c_int
    L.wb_trip_choice.argtypes = [ctypes.c_char_p, ctypes.c_uint32]
    fib = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fibonacci.wasm"), "rb").read()
    want = {"c1": (fib, 0), "c2": (W.blake3_wasm(), 0), "c3": (W.qsort_wasm(), 1),
            "c4": (W.collatz_wasm(), 1), "c5": (W.mandel_wasm(), 0)}
    got = {k: L.wb_trip_choice(w, len(w)) for k, (w, _) in want.items()}
    assert got == {k: v for k, (_, v) in want.items()}
