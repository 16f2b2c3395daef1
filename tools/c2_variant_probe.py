"""Probe: where C2's wait time goes. Times the C2 kernel (64K instances x run(iid, 1000))
for variants of the compression body with the same VALU work: cv loaded from an address
the loop never stores (no store->load dependence), cv from a local (no cv loads), block
words as constants (no block loads). Debug aid, not a test."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from wasmedge_amd import batch, workloads as W
from wasmedge_amd.wat import assemble

base = W.blake3_wat()
cv = ["local.get $cv i32.load offset=%d local.set $v%d" % (4 * k, k) for k in range(8)]
blk = ["local.get $blk i32.load offset=%d local.set $m%d" % (4 * k, k) for k in range(16)]
assert all(s in base for s in cv + blk)


def sub(src, pairs):
    for a, b in pairs:
        src = src.replace(a, b)
    return src


variants = {
    "base": base,
    "nodep": sub(base, [(cv[k], "local.get $blk i32.load offset=%d local.set $v%d" % (64 + 4 * k, k))
                        for k in range(8)]),
    "nocv": sub(base, [(cv[k], "local.get $ctr_lo local.set $v%d" % k) for k in range(8)]),
    "noblk": sub(base, [(blk[k], "i32.const %d local.set $m%d" % (k * 77 + 5, k)) for k in range(16)]),
}
variants["none"] = sub(variants["nocv"], [(blk[k], "i32.const %d local.set $m%d" % (k * 77 + 5, k))
                                          for k in range(16)])
c0 = base.index("(call $compress (i32.const 256)")
c1 = base.index("(br_if $chain")
loop_call = base[c0:c1]
for u in (2, 4):   # the chain loop's body compresses u times per trip (iters % u == 0)
    variants["unroll%d" % u] = base.replace(loop_call, loop_call * u)
n, iters = 65536, 1000
only = sys.argv[1:] or list(variants)
# NAME@VAR=VAL: the variant with an environment knob set while its context compiles
for spec in only:
    name, _, env = spec.partition("@")
    saved = dict(os.environ)
    if env:
        k, _, v = env.partition("=")
        os.environ[k] = v
    wasm = assemble(variants[name])
    ctx = batch.BatchContext(wasm, n)
    ctx.set_args("run", batch.make_values([[i, iters] for i in range(n)], [0x7F, 0x7F]))
    ctx.reset(); ctx.run()
    ks = []
    for _ in range(3):
        ctx.reset(timed=False)
        ks.append(ctx.run())
    _, st, cnt = ctx.results(1)
    print("%-6s kernel %.3f ms  instr/lane %d  traps %d" % (spec, 1e3 * min(ks), int(cnt[0]),
                                                         int((st != 0).sum())), flush=True)
    ctx.close()
    os.environ.clear()
    os.environ.update(saved)
