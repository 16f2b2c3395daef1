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
    rec, bpi = bench.cpu_baseline(wasm, func, build_rows, ptypes, 0.5, 2, gpu, name.upper())
    assert rec["kind"] == "port" and rec["cores"] == 2 and rec["value"] > 0
    assert bpi > 0
    # a wrong result for any sampled instance must fail the run loudly
    gpu["counts"] = gpu["counts"].copy()
    gpu["counts"][0] += 1
    with pytest.raises(SystemExit):
        bench.cpu_baseline(wasm, func, build_rows, ptypes, 0.5, 2, gpu, name.upper())
