# r06 zq: same-build profiles after the every-16th-trip convergence test: C3 on memory 1, C3 grown
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zq; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=170
step prof_c3x 800 bash $R/tools/prof_bench.sh gpurun_out/r06zq/c3x --workload c3x
step prof_c3grow 800 bash $R/tools/prof_bench.sh gpurun_out/r06zq/c3grow --workload c3grow
echo all done
