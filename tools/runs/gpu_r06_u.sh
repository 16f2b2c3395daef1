# r06 u: same-build rocprofv3 profile of C3 on memory 1 (c3x, 64K x 1 MiB)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06u; mkdir -p $O
export PROF_TIMEOUT=170
timeout -k 10 1150 bash $R/tools/prof_bench.sh gpurun_out/r06u/c3x --workload c3x > $O/prof_c3x.log 2>&1 && echo c3x profiled
