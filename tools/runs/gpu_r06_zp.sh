# r06 zp: the convergence test every 16th trip: trip parity, then same-build profiles of C4, mt19937, C3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zp; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_xmem_jit.py -m gpu -v --timeout 300 --timeout-method thread
export PROF_TIMEOUT=170
step prof_c4 200 bash $R/tools/prof_bench.sh gpurun_out/r06zp/c4 --workload c4
step prof_mt 300 bash $R/tools/prof_bench.sh gpurun_out/r06zp/mt --workload mt
step prof_c3 800 bash $R/tools/prof_bench.sh gpurun_out/r06zp/c3 --workload c3
echo all done
