"""The interleave granule chosen at run time (batch_api.cpp layout_trial).

A module whose load/store addresses may differ between instances (Program::divergent_mem)
starts with 128-byte granules; its first run is a warm-up, its second measures wasm
instructions per kernel second, the next Reset switches to 4-byte words, the third run
measures again, and the faster layout stays (4-byte only when >= 10% faster), the switch
back happening at the following Reset. mt19937 (test/thread/ThreadTest.cpp:31-150) keeps its state index in memory, so the
static analysis calls it divergent although every lane walks the same addresses: it ends
on 4-byte words (1.7e12 instr/s against 1.1e12 at 128, DESIGN.md "Linear memory"). Results
never depend on the layout: every run here is bit-exact against the oracle.
"""
import oracle_py as O
import pytest

from conftest import golden
from helpers import compare, oracle_run

I32, I64 = 0x7F, 0x7E


def _runs(wasm, func, rows, ptypes, rtypes, nruns, **kw):
    from wasmedge_amd import batch
    ctx = batch.BatchContext(wasm, len(rows), **kw)
    out = []
    try:
        vals = batch.make_values(rows, ptypes)
        for k in range(nruns):
            if k:
                ctx.reset()
            rets, st, cnt = ctx.execute(func, vals, len(rtypes))
            ints = batch.ret_ints(rets)
            got = [[int(x) for x in ints[i]] if st[i] == 0 else [] for i in range(len(rows))]
            out.append((ctx.memory_granule(), got, st, cnt, ctx.memory_hash()))
    finally:
        ctx.close()
    return out


@pytest.mark.gpu
def test_gpu_mt19937_settles_on_words(built):
    """mt19937 with per-instance seeds: 128-byte granules on the first two runs (warm-up,
    measured), 4-byte words from the third on (the trial keeps them), every run bit-exact."""
    wasm = golden("mt19937.wasm")
    n = 16384
    rows = [[0, 5489 + i, 20000] for i in range(n)]
    idx = list(range(0, n, 509)) + [n - 1]
    ref = oracle_run(O.Module(wasm), "mt19937", [rows[i] for i in idx])
    out = _runs(wasm, "mt19937", rows, [I32, I64, I64], [I64], 5)
    for k, (g, got, st, cnt, h) in enumerate(out):
        assert compare(ref, [got[i] for i in idx], st[idx], cnt[idx], h[idx], [I64]) == [], k
    # (4-byte words: every lane's state index is the same word)
    assert [o[0] for o in out] == [128, 128, 4, 4, 4]


@pytest.mark.gpu
def test_gpu_trial_off_and_explicit_granule(built, monkeypatch):
    """WB_GRANULE_TRIAL=0 and an explicit MemoryGranule keep the layout fixed."""
    wasm = golden("mt19937.wasm")
    rows = [[0, 7 + i, 500] for i in range(256)]
    assert [o[0] for o in _runs(wasm, "mt19937", rows, [I32, I64, I64], [I64], 3, memory_granule=16)] == [16] * 3
    monkeypatch.setenv("WB_GRANULE_TRIAL", "0")
    assert [o[0] for o in _runs(wasm, "mt19937", rows, [I32, I64, I64], [I64], 3)] == [128] * 3


@pytest.mark.gpu
def test_gpu_qsort_trial_exact(built):
    """C3's quicksort through the trial (whichever layout wins): bit-exact on every run,
    memory hashes included, across both re-layouts."""
    from wasmedge_amd import workloads as W
    wasm = W.qsort_wasm()
    rows = [[i, 2048] for i in range(4096)]
    idx = list(range(0, 4096, 97))
    ref = oracle_run(O.Module(wasm), "sort", [rows[i] for i in idx])
    out = _runs(wasm, "sort", rows, [I32, I32], [I32], 5)
    for k, (g, got, st, cnt, h) in enumerate(out):
        assert g in (4, 128)
        assert compare(ref, [got[i] for i in idx], st[idx], cnt[idx], h[idx], [I32]) == [], k
    assert out[0][0] == 128 and out[1][0] == 128 and out[2][0] == 4 and out[3][0] == out[4][0]
