"""Debug probe: minimal load-scan loops (jit.cpp scan blocks) on the GPU vs the oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle_py as O
from wasmedge_amd import batch
from wasmedge_amd.wat import assemble
d = sys.argv[1] if len(sys.argv) > 1 else "add"
off = int(sys.argv[2]) if len(sys.argv) > 2 else 4
wat = r"""
(module (memory 1)
 (func (export "run") (param $s i32) (result i64)
   (local $x i32) (local $p i32) (local $k i32)
   (loop $f (i32.store (i32.shl (local.get $k) (i32.const 2))
              (i32.and (i32.add (i32.mul (local.get $k) (i32.const 7919)) (local.get $s)) (i32.const 255)))
            (local.set $k (i32.add (local.get $k) (i32.const 1)))
            (br_if $f (i32.lt_u (local.get $k) (i32.const 16384))))
   (local.set $x (i32.and (i32.add (i32.const 1024) (i32.mul (local.get $s) (i32.const 52))) (i32.const 0xFFFC)))
   (local.set $p (i32.and (local.get $s) (i32.const 63)))
   (loop $l (local.set $x (i32.%s (local.get $x) (i32.const 4)))
            (br_if $l (i32.gt_u (i32.load offset=%d (local.get $x)) (local.get $p))))
   (i64.extend_i32_u (local.get $x))))
""" % (d, off)
wasm = assemble(wat)
n = 256
rows = [[i * 97 + 13] for i in range(n)]
m = O.Module(wasm)
ref = [m.run("run", r) for r in rows]
ctx = batch.BatchContext(wasm, n)
rets, st, cnt = ctx.execute("run", batch.make_values(rows, [batch.I32]), 1)
vals = batch.ret_ints(rets)
ctx.close()
bad = 0
for i in range(n):
    code, rv, rc, _ = ref[i]
    if int(st[i]) != code or int(cnt[i]) != rc or (code == 0 and int(vals[i][0]) != rv[0]):
        bad += 1
        if bad <= 6:
            print("lane %d: st %d/%d x %d/%d count %d/%d" % (i, int(st[i]), code, int(vals[i][0]), rv[0] if rv else -1, int(cnt[i]), rc))
print(d, off, "bad", bad, "of", n)
