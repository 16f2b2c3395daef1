# r06 st: same-build rocprofv3 profiles at HEAD: C1, mt19937, tail calls, then C3 (64K x 1 MiB)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06s; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=170
step prof_c1 300 bash $R/tools/prof_bench.sh gpurun_out/r06s/c1 --workload c1
step prof_mt 300 bash $R/tools/prof_bench.sh gpurun_out/r06s/mt --workload mt
step prof_tail 300 bash $R/tools/prof_bench.sh gpurun_out/r06s/tail --workload tail
step prof_c3 800 bash $R/tools/prof_bench.sh gpurun_out/r06s/c3 --workload c3
echo all done
