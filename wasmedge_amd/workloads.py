"""The config modules of BASELINE.json, authored in WAT and assembled by wat.py.

  C1 fib       tools/wasmedge/examples/fibonacci.wasm (the reference's own file, in
               tests/golden/) -- recursive i32, no memory
  C2 blake3    BLAKE3 compression restated in wasm (thirdparty/blake3/blake3_portable.c:
               g/round_fn/compress_pre, MSG_SCHEDULE blake3_impl.h:77-85), chained `iters`
               times over per-instance splitmix64 input; plus a single-chunk `blake3`
               export pinned by test/aot/AOTBlake3Test.cpp's Empty/Small/Large KATs
  C3 qsort     per-instance xorshift32 array in linear memory, recursive quicksort
               (Hoare partition, recurse on the smaller side), weighted checksum
  C4 collatz   br_table state machine over i64 Collatz steps with per-lane traps
               (unreachable / div-by-zero / out-of-bounds load) on chosen instance ids
  C5 mandel    f64x2 SIMD128 Mandelbrot 8x8-pixel tiles (docs/simd.md kernel shape),
               pixel bytes stored to memory, 64-bit inside-mask returned
"""
from .wat import assemble

IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
      0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
MSG_SCHEDULE = [
    [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15],
    [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8],
    [3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1],
    [10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6],
    [12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4],
    [9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7],
    [11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13],
]

# ---------------------------------------------------------------------------- C2
BLAKE3_CV = 256      # chaining value (32 B) used by run()
BLAKE3_BLOCK = 288   # message block (64 B) used by run()


def _g(a, b, c, d, x, y):
    """One BLAKE3 G mixing step (blake3_portable.c:12-21) as flat wasm."""
    out = []

    def add3(dst, s1, s2):
        out.append("local.get $v%d local.get $v%d i32.add local.get $m%d i32.add local.set $v%d"
                   % (dst, s1, s2, dst))

    def xrot(dst, s, r):
        out.append("local.get $v%d local.get $v%d i32.xor i32.const %d i32.rotr local.set $v%d"
                   % (dst, s, r, dst))

    def add2(dst, s):
        out.append("local.get $v%d local.get $v%d i32.add local.set $v%d" % (dst, s, dst))

    add3(a, b, x); xrot(d, a, 16); add2(c, d); xrot(b, c, 12)
    add3(a, b, y); xrot(d, a, 8); add2(c, d); xrot(b, c, 7)
    return "\n".join(out)


def _compress_body():
    lines = []
    for k in range(16):
        lines.append("local.get $blk i32.load offset=%d local.set $m%d" % (4 * k, k))
    for k in range(8):
        lines.append("local.get $cv i32.load offset=%d local.set $v%d" % (4 * k, k))
    for k in range(4):
        lines.append("i32.const %d local.set $v%d" % (IV[k] - (1 << 32) if IV[k] >= 1 << 31 else IV[k], 8 + k))
    lines.append("local.get $ctr_lo local.set $v12")
    lines.append("local.get $ctr_hi local.set $v13")
    lines.append("local.get $blen local.set $v14")
    lines.append("local.get $flags local.set $v15")
    for r in range(7):
        s = MSG_SCHEDULE[r]
        lines.append(_g(0, 4, 8, 12, s[0], s[1]))
        lines.append(_g(1, 5, 9, 13, s[2], s[3]))
        lines.append(_g(2, 6, 10, 14, s[4], s[5]))
        lines.append(_g(3, 7, 11, 15, s[6], s[7]))
        lines.append(_g(0, 5, 10, 15, s[8], s[9]))
        lines.append(_g(1, 6, 11, 12, s[10], s[11]))
        lines.append(_g(2, 7, 8, 13, s[12], s[13]))
        lines.append(_g(3, 4, 9, 14, s[14], s[15]))
    for k in range(8):   # output cv = v[k] ^ v[k+8]
        lines.append("local.get $out local.get $v%d local.get $v%d i32.xor i32.store offset=%d"
                     % (k, k + 8, 4 * k))
    return "\n".join(lines)


def blake3_wat():
    locs = " ".join("(local $v%d i32)" % k for k in range(16)) + " " + \
        " ".join("(local $m%d i32)" % k for k in range(16))
    iv_bytes = "".join("\\%02x" % b for w in IV for b in w.to_bytes(4, "little"))
    return r"""
(module
  (memory (export "memory") 1)
  (data (i32.const 0) "%s")
  ;; compress_pre + compress_in_place output (blake3_portable.c:30-113): out[0..8) = v[k]^v[k+8]
  (func $compress (param $cv i32) (param $blk i32) (param $ctr_lo i32) (param $ctr_hi i32)
                  (param $blen i32) (param $flags i32) (param $out i32)
    %s
    %s)
  ;; single-chunk BLAKE3 hash of mem[ptr, ptr+len), len <= 1024, 32 bytes to out.
  ;; blocks are copied into a zero-padded scratch block at 128; cv lives at 64.
  (func (export "blake3") (param $ptr i32) (param $len i32) (param $out i32)
    (local $off i32) (local $n i32) (local $flags i32) (local $k i32)
    (memory.copy (i32.const 64) (i32.const 0) (i32.const 32))
    (block $done
      (loop $blocks
        (local.set $n (i32.sub (local.get $len) (local.get $off)))
        (if (i32.gt_u (local.get $n) (i32.const 64)) (then (local.set $n (i32.const 64))))
        (memory.fill (i32.const 128) (i32.const 0) (i32.const 64))
        (memory.copy (i32.const 128) (i32.add (local.get $ptr) (local.get $off)) (local.get $n))
        (local.set $flags (i32.const 0))
        (if (i32.eqz (local.get $off)) (then (local.set $flags (i32.const 1))))
        (if (i32.ge_u (i32.add (local.get $off) (i32.const 64)) (local.get $len))
          (then (local.set $flags (i32.or (local.get $flags) (i32.const 10)))))
        (call $compress (i32.const 64) (i32.const 128) (i32.const 0) (i32.const 0)
                        (local.get $n) (local.get $flags) (i32.const 64))
        (local.set $off (i32.add (local.get $off) (i32.const 64)))
        (br_if $blocks (i32.lt_u (local.get $off) (local.get $len)))))
    (memory.copy (local.get $out) (i32.const 64) (i32.const 32)))
  ;; C2 workload: per-instance input from splitmix64(iid ^ 0x5EED) -> cv (32 B) + block
  ;; (64 B); `iters` chained compressions (counter = iteration); returns cv[0].
  (func (export "run") (param $iid i32) (param $iters i32) (result i32)
    (local $s i64) (local $z i64) (local $k i32) (local $i i32)
    (local.set $s (i64.extend_i32_u (i32.xor (local.get $iid) (i32.const 0x5EED))))
    (loop $fill
      (local.set $s (i64.add (local.get $s) (i64.const 0x9E3779B97F4A7C15)))
      (local.set $z (local.get $s))
      (local.set $z (i64.mul (i64.xor (local.get $z) (i64.shr_u (local.get $z) (i64.const 30)))
                             (i64.const 0xBF58476D1CE4E5B9)))
      (local.set $z (i64.mul (i64.xor (local.get $z) (i64.shr_u (local.get $z) (i64.const 27)))
                             (i64.const 0x94D049BB133111EB)))
      (local.set $z (i64.xor (local.get $z) (i64.shr_u (local.get $z) (i64.const 31))))
      (i64.store offset=%d (i32.shl (local.get $k) (i32.const 3)) (local.get $z))
      (local.set $k (i32.add (local.get $k) (i32.const 1)))
      (br_if $fill (i32.lt_u (local.get $k) (i32.const 12))))
    (block $end
      (br_if $end (i32.eqz (local.get $iters)))
      (loop $chain
        (call $compress (i32.const %d) (i32.const %d) (local.get $i) (i32.const 0)
                        (i32.const 64) (i32.const 0) (i32.const %d))
        (local.set $i (i32.add (local.get $i) (i32.const 1)))
        (br_if $chain (i32.lt_u (local.get $i) (local.get $iters)))))
    (i32.load (i32.const %d)))
)
""" % (iv_bytes, locs, _compress_body(), BLAKE3_CV, BLAKE3_CV, BLAKE3_BLOCK, BLAKE3_CV, BLAKE3_CV)


def blake3_wasm():
    return assemble(blake3_wat())


# ---------------------------------------------------------------------------- C3
QSORT_BASE = 65536


def qsort_wat(pages=17):
    return r"""
(module
  (memory (export "memory") %d)
  ;; Hoare-partition quicksort on i32 a[lo..hi] (byte addresses), recursing on the
  ;; smaller side and looping on the larger (depth <= log2 n).
  (func $qsort (param $lo i32) (param $hi i32)
    (local $i i32) (local $j i32) (local $p i32) (local $t i32)
    (block $out
      (loop $again
        (br_if $out (i32.ge_u (local.get $lo) (local.get $hi)))
        ;; pivot = middle element
        (local.set $p (i32.load (i32.add (local.get $lo)
          (i32.and (i32.shr_u (i32.sub (local.get $hi) (local.get $lo)) (i32.const 1))
                   (i32.const -4)))))
        (local.set $i (i32.sub (local.get $lo) (i32.const 4)))
        (local.set $j (i32.add (local.get $hi) (i32.const 4)))
        (block $parted
          (loop $part
            (loop $li
              (local.set $i (i32.add (local.get $i) (i32.const 4)))
              (br_if $li (i32.lt_s (i32.load (local.get $i)) (local.get $p))))
            (loop $lj
              (local.set $j (i32.sub (local.get $j) (i32.const 4)))
              (br_if $lj (i32.gt_s (i32.load (local.get $j)) (local.get $p))))
            (br_if $parted (i32.ge_u (local.get $i) (local.get $j)))
            (local.set $t (i32.load (local.get $i)))
            (i32.store (local.get $i) (i32.load (local.get $j)))
            (i32.store (local.get $j) (local.get $t))
            (br $part)))
        ;; [lo, j] and [j+4, hi]: recurse on the smaller side
        (if (i32.lt_u (i32.sub (local.get $j) (local.get $lo))
                      (i32.sub (local.get $hi) (local.get $j)))
          (then
            (call $qsort (local.get $lo) (local.get $j))
            (local.set $lo (i32.add (local.get $j) (i32.const 4))))
          (else
            (call $qsort (i32.add (local.get $j) (i32.const 4)) (local.get $hi))
            (local.set $hi (local.get $j))))
        (br $again))))
  ;; C3 workload: fill n i32 at 65536 from xorshift32(iid*2654435761+1), sort, and
  ;; return sum(a[k]*(k+1)) mod 2^32.
  (func (export "sort") (param $iid i32) (param $n i32) (result i32)
    (local $x i32) (local $k i32) (local $sum i32) (local $end i32)
    (local.set $x (i32.add (i32.mul (local.get $iid) (i32.const 2654435761)) (i32.const 1)))
    (if (i32.eqz (local.get $x)) (then (local.set $x (i32.const 1))))
    (local.set $end (i32.add (i32.const %d) (i32.shl (local.get $n) (i32.const 2))))
    (local.set $k (i32.const %d))
    (block $filled
      (loop $fill
        (br_if $filled (i32.ge_u (local.get $k) (local.get $end)))
        (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 13))))
        (local.set $x (i32.xor (local.get $x) (i32.shr_u (local.get $x) (i32.const 17))))
        (local.set $x (i32.xor (local.get $x) (i32.shl (local.get $x) (i32.const 5))))
        (i32.store (local.get $k) (local.get $x))
        (local.set $k (i32.add (local.get $k) (i32.const 4)))
        (br $fill)))
    (if (local.get $n)
      (then (call $qsort (i32.const %d) (i32.sub (local.get $end) (i32.const 4)))))
    (local.set $k (i32.const 0))
    (block $summed
      (loop $sum
        (br_if $summed (i32.ge_u (local.get $k) (local.get $n)))
        (local.set $sum (i32.add (local.get $sum)
          (i32.mul (i32.load offset=%d (i32.shl (local.get $k) (i32.const 2)))
                   (i32.add (local.get $k) (i32.const 1)))))
        (local.set $k (i32.add (local.get $k) (i32.const 1)))
        (br $sum)))
    (local.get $sum))
)
""" % (pages, QSORT_BASE, QSORT_BASE, QSORT_BASE, QSORT_BASE)


def qsort_wasm(pages=17):
    return assemble(qsort_wat(pages))


def qsort_grow_wat():
    """C3's quicksort in a module that starts with ONE page and grows to what the sort
    needs (1 + ceil((65536 + 4n) / 65536) pages) before filling it -- the allocator-driven
    shape (a Rust/C module's heap) whose pages all come from memory.grow. No declared max:
    the reference's default limit (65536) applies."""
    src = qsort_wat(1)
    old = "    (local.set $x (i32.add (i32.mul (local.get $iid) (i32.const 2654435761)) (i32.const 1)))"
    assert old in src
    grow = ("    (drop (memory.grow (i32.sub (i32.shr_u (i32.add (i32.const %d) (i32.add (i32.shl (local.get $n)"
            " (i32.const 2)) (i32.const 65535))) (i32.const 16)) (memory.size))))\n" % QSORT_BASE)
    return src.replace(old, grow + old)


def qsort_grow_wasm():
    return assemble(qsort_grow_wat())


def qsort_x_wat(pages=17):
    """C3's quicksort with its array on memory 1 (the MultiMemories proposal): memory 0 is
    a one-page memory nothing touches, and every load and store names memory 1 -- the same
    program, instruction for instruction, on a memory past the first (the
    compiled XLD / XST against C3's memory-0 accesses)."""
    src = qsort_wat(pages)
    old = '  (memory (export "memory") %d)' % pages
    assert old in src
    src = src.replace(old, "  (memory $m0 1)\n  (memory $m1 %d)" % pages)
    for op in ("i32.load", "i32.store"):
        src = src.replace("(%s " % op, "(%s $m1 " % op)
    return src


def qsort_x_wasm(pages=17):
    return assemble(qsort_x_wat(pages))


# ---------------------------------------------------------------------------- C4
def collatz_wat():
    return r"""
(module
  (memory (export "memory") 1)
  ;; C4 workload: n = iid*7919 + 1 (i64). A 4-state br_table machine
  ;; (0 = check, 1 = even, 2 = odd, 3 = done) steps Collatz until n == 1 or `limit`
  ;; steps. Per-lane traps: iid % 97 == 0 -> unreachable, iid % 89 == 0 -> i32.div_u
  ;; by zero, iid % 83 == 0 -> i32.load at 0xFFFFFFF0 (out of bounds).
  ;; Returns steps + 1000003 * (max value mod 1000).
  (func (export "collatz") (param $iid i32) (param $limit i32) (result i32)
    (local $n i64) (local $state i32) (local $steps i32) (local $mx i64)
    (local.set $n (i64.add (i64.mul (i64.extend_i32_u (local.get $iid)) (i64.const 7919))
                           (i64.const 1)))
    (local.set $mx (local.get $n))
    (block $done
      (loop $machine
        (block $odd
          (block $even
            (block $check
              (br_table $check $even $odd $done (local.get $state)))
            ;; check
            (if (i64.le_u (local.get $n) (i64.const 1)) (then (br $done)))
            (if (i32.ge_u (local.get $steps) (local.get $limit)) (then (br $done)))
            (local.set $state (i32.add (i32.const 1) (i32.wrap_i64 (i64.and (local.get $n) (i64.const 1)))))
            (br $machine))
          ;; even
          (local.set $n (i64.shr_u (local.get $n) (i64.const 1)))
          (local.set $steps (i32.add (local.get $steps) (i32.const 1)))
          (local.set $state (i32.const 0))
          (br $machine))
        ;; odd
        (local.set $n (i64.add (i64.mul (local.get $n) (i64.const 3)) (i64.const 1)))
        (if (i64.gt_u (local.get $n) (local.get $mx)) (then (local.set $mx (local.get $n))))
        (local.set $steps (i32.add (local.get $steps) (i32.const 1)))
        (local.set $state (i32.const 0))
        (br $machine)))
    (if (i32.eqz (i32.rem_u (local.get $iid) (i32.const 97))) (then unreachable))
    (if (i32.eqz (i32.rem_u (local.get $iid) (i32.const 89)))
      (then (drop (i32.div_u (local.get $steps) (i32.const 0)))))
    (if (i32.eqz (i32.rem_u (local.get $iid) (i32.const 83)))
      (then (drop (i32.load (i32.const 0xFFFFFFF0)))))
    (i32.add (local.get $steps)
             (i32.mul (i32.const 1000003) (i32.wrap_i64 (i64.rem_u (local.get $mx) (i64.const 1000))))))
)
"""


def collatz_wasm():
    return assemble(collatz_wat())


# ---------------------------------------------------------------------------- C5
def mandel_wat():
    return r"""
(module
  (memory (export "memory") 1)
  ;; C5 workload (docs/simd.md:12-130 kernel shape): tile `iid` of a W x H image split
  ;; into 8x8-pixel tiles; c in [-1.5,0.5] x [-1,1]; two pixels per f64x2 lane pair;
  ;; `iters` iterations with limit^2 = 4. Each pixel's escape iteration count (byte) is
  ;; stored at 64*row... (tile-local, offset 0); returns the 64-bit inside mask.
  (func (export "tile") (param $iid i32) (param $w i32) (param $iters i32) (result i64)
    (local $tx i32) (local $ty i32) (local $py i32) (local $px i32) (local $k i32)
    (local $cr v128) (local $ci v128) (local $zr v128) (local $zi v128) (local $zr2 v128)
    (local $zi2 v128) (local $cnt v128) (local $act v128) (local $mask i64)
    (local $dx f64) (local $dy f64)
    (local.set $tx (i32.rem_u (local.get $iid) (i32.shr_u (local.get $w) (i32.const 3))))
    (local.set $ty (i32.div_u (local.get $iid) (i32.shr_u (local.get $w) (i32.const 3))))
    (local.set $dx (f64.div (f64.const 2.0) (f64.convert_i32_u (local.get $w))))
    (local.set $dy (local.get $dx))
    (loop $rows
      (local.set $px (i32.const 0))
      (loop $cols
        ;; two pixels: x = tx*8+px, tx*8+px+1
        (local.set $cr (f64x2.add (f64x2.splat (f64.const -1.5))
          (f64x2.mul (f64x2.splat (local.get $dx))
            (f64x2.replace_lane 1
              (f64x2.splat (f64.convert_i32_u (i32.add (i32.shl (local.get $tx) (i32.const 3)) (local.get $px))))
              (f64.convert_i32_u (i32.add (i32.add (i32.shl (local.get $tx) (i32.const 3)) (local.get $px)) (i32.const 1)))))))
        (local.set $ci (f64x2.splat (f64.add (f64.const -1.0)
          (f64.mul (local.get $dy) (f64.convert_i32_u (i32.add (i32.shl (local.get $ty) (i32.const 3)) (local.get $py)))))))
        (local.set $zr (v128.const i64x2 0 0))
        (local.set $zi (v128.const i64x2 0 0))
        (local.set $cnt (v128.const i64x2 0 0))
        (local.set $k (i32.const 0))
        (block $esc
          (loop $it
            (local.set $zr2 (f64x2.mul (local.get $zr) (local.get $zr)))
            (local.set $zi2 (f64x2.mul (local.get $zi) (local.get $zi)))
            (local.set $act (f64x2.le (f64x2.add (local.get $zr2) (local.get $zi2))
                                      (f64x2.splat (f64.const 4.0))))
            (br_if $esc (i32.eqz (v128.any_true (local.get $act))))
            (local.set $cnt (i64x2.sub (local.get $cnt) (local.get $act)))
            (local.set $zi (f64x2.add (f64x2.mul (f64x2.mul (local.get $zr) (local.get $zi))
                                                 (f64x2.splat (f64.const 2.0)))
                                      (local.get $ci)))
            (local.set $zr (f64x2.add (f64x2.sub (local.get $zr2) (local.get $zi2)) (local.get $cr)))
            (local.set $k (i32.add (local.get $k) (i32.const 1)))
            (br_if $it (i32.lt_u (local.get $k) (local.get $iters)))))
        ;; store the two counts as bytes, fold 'inside' bits into the mask
        (i32.store8 (i32.add (i32.shl (local.get $py) (i32.const 3)) (local.get $px))
                    (i32.wrap_i64 (i64x2.extract_lane 0 (local.get $cnt))))
        (i32.store8 offset=1 (i32.add (i32.shl (local.get $py) (i32.const 3)) (local.get $px))
                    (i32.wrap_i64 (i64x2.extract_lane 1 (local.get $cnt))))
        (local.set $mask (i64.or (local.get $mask)
          (i64.shl (i64.extend_i32_u (i32x4.bitmask (i64x2.eq (local.get $cnt)
                      (i64x2.splat (i64.extend_i32_u (local.get $iters))))))
                   (i64.extend_i32_u (i32.add (i32.shl (local.get $py) (i32.const 3)) (local.get $px))))))
        (local.set $px (i32.add (local.get $px) (i32.const 2)))
        (br_if $cols (i32.lt_u (local.get $px) (i32.const 8))))
      (local.set $py (i32.add (local.get $py) (i32.const 1)))
      (br_if $rows (i32.lt_u (local.get $py) (i32.const 8))))
    (local.get $mask))
)
"""


def mandel_wasm():
    return assemble(mandel_wat())


# ----------------------------------------------------------------- tail calls (not a config)
def tail_wat():
    return r"""
(module
  ;; Tail recursion with the TailCall proposal (return_call / return_call_indirect): a
  ;; countdown accumulating a hash, which every 16th step calls a mutually tail-recursive
  ;; even/odd pair over the low bits, one of them through a table. Frames never grow:
  ;; run(iid, n) takes n + iid mod 13 outer steps.
  (type $t (func (param i32 i32) (result i32)))
  (table 2 funcref)
  (elem (i32.const 0) $even $odd)
  (func $even (type $t) (param $k i32) (param $acc i32) (result i32)
    (if (result i32) (i32.eqz (local.get $k))
      (then (i32.add (local.get $acc) (i32.const 1)))
      (else (return_call_indirect (type $t) (i32.sub (local.get $k) (i32.const 1))
                                  (i32.xor (local.get $acc) (local.get $k)) (i32.const 1)))))
  (func $odd (type $t) (param $k i32) (param $acc i32) (result i32)
    (if (result i32) (i32.eqz (local.get $k))
      (then (local.get $acc))
      (else (return_call $even (i32.sub (local.get $k) (i32.const 1))
                               (i32.add (local.get $acc) (local.get $k))))))
  (func $loop (param $n i32) (param $acc i32) (result i32)
    (if (result i32) (i32.eqz (local.get $n))
      (then (local.get $acc))
      (else
        (if (i32.eqz (i32.and (local.get $n) (i32.const 15)))
          (then (local.set $acc (call $even (i32.and (local.get $acc) (i32.const 7)) (local.get $acc)))))
        (return_call $loop (i32.sub (local.get $n) (i32.const 1))
                           (i32.add (i32.mul (local.get $acc) (i32.const 31)) (local.get $n))))))
  (func (export "run") (param $iid i32) (param $n i32) (result i32)
    (return_call $loop (i32.add (local.get $n) (i32.rem_u (local.get $iid) (i32.const 13)))
                       (local.get $iid))))
"""


def tail_wasm():
    return assemble(tail_wat())


WORKLOADS = {
    "blake3": (blake3_wasm, "run"),
    "qsort": (qsort_wasm, "sort"),
    "collatz": (collatz_wasm, "collatz"),
    "mandel": (mandel_wasm, "tile"),
}


def blake3_kat_wasm(msg):
    """blake3 module + the message at 1024 and an export kat(word) that hashes it
    (single chunk) and returns output word `word` -- checks the wasm compression against
    test/aot/AOTBlake3Test.cpp:31-77."""
    data = "".join("\\%02x" % b for b in msg)
    extra = r"""
  (data (i32.const 1024) "%s")
  (func (export "kat") (param $word i32) (result i32)
    (call 1 (i32.const 1024) (i32.const %d) (i32.const 512))
    (i32.load offset=512 (i32.shl (local.get $word) (i32.const 2))))
)
""" % (data, len(msg))
    src = blake3_wat().rstrip()
    assert src.endswith(")")
    return assemble(src[:-1] + extra)
