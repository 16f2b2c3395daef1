# r06 zw: the trips left only when no lane is in them (exit threshold k = 6): trip parity,
# same-build profile of C4
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zw; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_xmem_jit.py tests/test_hostcall.py tests/test_metering.py -m gpu -v --timeout 300 --timeout-method thread
export PROF_TIMEOUT=170
step prof_c4 200 bash $R/tools/prof_bench.sh gpurun_out/r06zw/c4 --workload c4
echo all done
