# r06 u: same-build rocprofv3 profiles of C3 on memory 1 (c3x) and C3 grown from one page
# (c3grow), both 64K x 1 MiB
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06u; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=170
step prof_c3x 560 bash $R/tools/prof_bench.sh gpurun_out/r06u/c3x --workload c3x
step prof_c3grow 560 bash $R/tools/prof_bench.sh gpurun_out/r06u/c3grow --workload c3grow
echo all done
