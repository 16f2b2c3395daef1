# r05 t: closing rocprofv3 evidence at HEAD for C2, C4, C5 (256K), mt19937, the tail-call
# workload and C1 (kernel trace + stats, FETCH/WRITE, issue counts, wave-cycle split,
# exec-mask efficiency, VMEM latency)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05t; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=150
step prof_c2 600 bash $R/tools/prof_bench.sh gpurun_out/r05t/c2 --steps 5 --warmup 2
step prof_c4 600 bash $R/tools/prof_bench.sh gpurun_out/r05t/c4 --workload c4 --steps 5 --warmup 2
step prof_c5 600 bash $R/tools/prof_bench.sh gpurun_out/r05t/c5 --workload c5 --instances 262144 --steps 5 --warmup 2
step prof_mt 600 bash $R/tools/prof_bench.sh gpurun_out/r05t/mt --workload mt --steps 3 --warmup 3
step prof_tail 600 bash $R/tools/prof_bench.sh gpurun_out/r05t/tail --workload tail --steps 3 --warmup 2
step prof_c1 900 bash $R/tools/prof_bench.sh gpurun_out/r05t/c1 --workload c1 --steps 1 --warmup 1
