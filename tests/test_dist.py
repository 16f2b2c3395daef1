"""Multi-GPU path, rehearsed on CPU: bench.py shards instances by id across ranks with no
data-path collective; only the timing bracket (barrier + max over ranks) and the job-wide
instruction total (sum) cross ranks.  world_size 2 over gloo, 127.0.0.1 rendezvous."""
import os
import socket
import sys

import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    d = bench.Dist()
    d.init()
    d.barrier()
    ids = bench.shard_ids(d.rank, 1000)
    q.put((rank, d.max(float(rank + 1)), d.sum(float(len(ids))), int(ids[0]), int(ids[-1])))
    d.barrier()
    d.td.destroy_process_group()


def test_dist_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert [o[1] for o in out] == [2.0, 2.0]        # max over ranks
    assert [o[2] for o in out] == [2000.0, 2000.0]  # job-wide total
    assert out[0][3:] == (0, 999) and out[1][3:] == (1000, 1999)   # disjoint id shards


def test_single_rank_needs_no_process_group():
    import bench
    d = bench.Dist()
    d.init()
    assert d.td is None and d.max(3.0) == 3.0 and d.sum(2.0) == 2.0
    assert list(bench.shard_ids(0, 4)) == [0, 1, 2, 3]


def _run_bench(*argv):
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(argv),
                         env=env, capture_output=True, text=True, timeout=240)
    return out.returncode, [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]


def test_bench_launcher_default_is_the_metric_config():
    """`bench.py --gpus 2` with no other option measures the metric's configuration: the
    job's 64K instances split over the GPUs (strong scaling)."""
    rc, lines = _run_bench("--gpus", "2", "--dry-run")
    assert rc == 0 and len(lines) == 1
    exp = lines[0].pop("expected_speedup")
    assert lines[0] == {"dry_run": True, "n_gpus": 2, "scaling": "strong", "instances": 65536,
                        "first_id": 0, "last_id": 65535, "max_over_ranks": 2.0}
    assert exp["value"] == 1.0 and "1024 waves" in exp["basis"]
    rc, lines = _run_bench("--gpus", "2", "--dry-run", "--workload", "c5")
    assert rc == 0 and lines[0]["instances"] == 262144


def test_bench_launcher_spawns_ranks_weak():
    """`bench.py --gpus 2 --scaling weak` run directly spawns one worker per GPU through its
    own launcher (no torchrun); the ranks rendezvous on 127.0.0.1, shard by id and reduce."""
    rc, lines = _run_bench("--gpus", "2", "--dry-run", "--scaling", "weak", "--instances", "65536")
    assert rc == 0 and len(lines) == 1
    assert lines[0].pop("expected_speedup")["value"] == 2.0
    assert lines[0] == {"dry_run": True, "n_gpus": 2, "scaling": "weak", "instances": 131072,
                        "first_id": 0, "last_id": 131071, "max_over_ranks": 2.0}


def test_bench_launcher_strong_scaling_splits_the_job():
    rc, lines = _run_bench("--gpus", "2", "--dry-run", "--scaling", "strong", "--instances", "65536")
    assert rc == 0 and lines[0]["instances"] == 65536 and lines[0]["last_id"] == 65535


def test_bench_refuses_mismatched_world_size():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


def test_strong_shards_cover_the_job():
    import bench
    for world in (1, 2, 4, 8):
        ids = [bench.shard_ids(r, 65536, world, "strong") for r in range(world)]
        assert sum(len(x) for x in ids) == 65536
        assert all(int(a[-1]) + 1 == int(b[0]) for a, b in zip(ids, ids[1:]))


def test_bench_expected_speedup_at_8_gpus():
    """an N > 1 line states the speed-up its configuration can give, with
    the basis -- ~1x at 64K instances (1024 waves = one per SIMD of one GPU), up to 4x for
    C5's 256K, N under weak scaling."""
    import bench
    rc, lines = _run_bench("--gpus", "8", "--dry-run")
    assert rc == 0 and lines[0]["n_gpus"] == 8
    assert lines[0]["expected_speedup"]["value"] == 1.0
    rc, lines = _run_bench("--gpus", "8", "--dry-run", "--workload", "c5")
    assert rc == 0 and lines[0]["expected_speedup"]["value"] == 4.0
    assert bench.expected_speedup(65536, 8, "weak")["value"] == 8.0
    assert bench.expected_speedup(262144, 2, "strong")["value"] == 2.0
