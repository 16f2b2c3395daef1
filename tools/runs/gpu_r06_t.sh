# r06 t: same-build rocprofv3 profile of C3 at its configs[2] size (64K x 1 MiB)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06t; mkdir -p $O
export PROF_TIMEOUT=170
timeout -k 10 1150 bash $R/tools/prof_bench.sh gpurun_out/r06t/c3 --workload c3 > $O/prof_c3.log 2>&1 && echo c3 profiled
