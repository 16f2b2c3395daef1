# r05 m: C3 4K counters after the trip shortcuts (all passes of tools/prof_bench.sh)
R=$GRAFT_REPO_ROOT
PROF_TIMEOUT=200 bash $R/tools/prof_bench.sh gpurun_out/r05m_c3k --workload c3 --elements 4096 --steps 2 --warmup 3
