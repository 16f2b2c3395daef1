# r06 w: no bounds / alignment tests in the load-cache stage (LtF) for accesses at the
# cached (already window-checked) addresses: trip-mode parity, then C3 4K / 1 MiB / memory 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06w; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_xmem_jit.py -m gpu -v --timeout 300 --timeout-method thread
step c3k_new 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3k_old 200 env WB_TRIP_FWDCHK=0 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3 300 python bench.py --workload c3 --no-cpu-baseline
echo all done
