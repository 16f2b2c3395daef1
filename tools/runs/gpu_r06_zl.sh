# r06 zl: the trips' convergence test every 4th trip (WB_TRIP_CONV1=1: every trip): parity, A/B on C4, C3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zl; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_xmem_jit.py tests/test_jit.py tests/test_memgrow.py tests/test_layout.py tests/test_metering.py tests/test_scalar.py -m gpu -v --timeout 300 --timeout-method thread
step c4_4 200 python bench.py --workload c4 --no-cpu-baseline
step c4_1 200 env WB_TRIP_CONV1=1 python bench.py --workload c4 --no-cpu-baseline
step c4_4b 200 python bench.py --workload c4 --no-cpu-baseline
step c4_1b 200 env WB_TRIP_CONV1=1 python bench.py --workload c4 --no-cpu-baseline
step c3k_4 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3k_1 200 env WB_TRIP_CONV1=1 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3_4 300 python bench.py --workload c3 --no-cpu-baseline
step mt_4 300 python bench.py --workload mt --no-cpu-baseline
echo all done
