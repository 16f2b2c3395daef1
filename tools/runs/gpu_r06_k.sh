# r06 k: C4 counters at HEAD (trip batching + guards) for the scalar-overhead question
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 900 bash tools/prof_bench.sh gpurun_out/r06k_c4 --workload c4 && echo c4 profiled
