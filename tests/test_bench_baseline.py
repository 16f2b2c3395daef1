"""bench.py's cpu_baseline leg on CPU: the oracle sample of each config workload must be
checked bit for bit against the batched results (here the host emulator's, standing in
for the GPU's), traps included, and yield the C3 roofline's bytes per instruction."""
import os
import sys
import types

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import helpers  # noqa: E402


def _fake_gpu(wasm, func, rows, ptypes, rtype, max_pages=0):
    rets, st, cnt, h = helpers.emu_run(wasm, func, [list(map(int, r)) for r in rows],
                                       ptypes, [rtype], max_pages=max_pages)
    ret = np.array([(r[0] if r else 0) & 0xFFFFFFFFFFFFFFFF for r in rets], np.uint64)
    return {"counts": cnt, "hashes": h, "status": st, "ret": ret, "ret32": rtype == 0x7F}


@pytest.mark.parametrize("name,n,elements", [("c3", 64, 512), ("c4", 200, 0), ("c2", 32, 0)])
def test_cpu_baseline_checks_sample(name, n, elements):
    import bench
    args = types.SimpleNamespace(iters=3, elements=elements)
    wasm, func, build_rows, ptypes, _desc, _extra = bench.workload(name, args)
    rows = build_rows(np.arange(n, dtype=np.int64))
    gpu = _fake_gpu(wasm, func, rows, [0x7F] * len(ptypes), 0x7F,
                    max_pages=17 if name == "c3" else 0)
    if name == "c4":
        assert (gpu["status"] != 0).any()   # the sample covers per-lane traps
    rec, bpi, (ld, stb) = bench.cpu_baseline(wasm, func, build_rows, ptypes, 0.5, 2, gpu, name.upper())
    assert rec["kind"] == "port" and rec["cores"] == 2 and rec["value"] > 0
    assert bpi > 0 and ld > 0 and stb >= 0 and abs(ld + stb - bpi) < 1e-9 * bpi
    if name in ("c2", "c3"):
        assert stb > 0   # (C4 only loads)
    # a wrong result for any sampled instance must fail the run loudly
    gpu["counts"] = gpu["counts"].copy()
    gpu["counts"][0] += 1
    with pytest.raises(SystemExit):
        bench.cpu_baseline(wasm, func, build_rows, ptypes, 0.5, 2, gpu, name.upper())


def test_check_engine_fails_on_silent_fallback(monkeypatch):
    """A bench line must not silently measure the threaded core after a compile failure
    (VERDICT r4 item 6): 0 compiled runs exits non-zero unless WB_JIT=0 asked for it."""
    import bench
    monkeypatch.delenv("WB_JIT", raising=False)
    bench.check_engine("c2", 12, "compiled-runs+simt/vgpr-frames")
    with pytest.raises(SystemExit) as e:
        bench.check_engine("c2", 0, "threaded-core (compiled runs failed)", "hiprtc: boom")
    assert "0 compiled runs" in str(e.value) and "hiprtc: boom" in str(e.value)
    monkeypatch.setenv("WB_JIT", "0")
    bench.check_engine("c2", 0, "threaded-core/vgpr-frames")


def test_vary_ids_are_fresh_permutations():
    """--vary-args: every step gives every instance another id (C5: another tile of the
    4096^2 image, a permutation of the 262,144 tiles)."""
    import bench
    ids = np.arange(262144, dtype=np.int64)
    seen = [ids]
    for k in range(3):
        v = bench.vary_ids(ids, k, "c5")
        assert sorted(v.tolist()) == ids.tolist()
        assert all((v != s).all() for s in seen)
        seen.append(v)
    v = bench.vary_ids(np.arange(65536, dtype=np.int64), 0, "c2")
    assert (v != np.arange(65536)).all() and v.max() < (1 << 30)


def test_default_instances_are_the_metric_config():
    import bench
    assert bench.default_instances("c2") == 65536 and bench.default_instances("c3") == 65536
    assert bench.default_instances("c5") == 262144
