# r06 zg: compare-branch reuses VCC in trip transfers (WB_TRIP_CMPBR): parity, then A/B on C4; C3 4K, C3 1 MiB, mt19937
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zg; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_xmem_jit.py tests/test_jit.py tests/test_memgrow.py tests/test_layout.py tests/test_bulk.py tests/test_scalar.py -m gpu -v --timeout 300 --timeout-method thread
step c4_on 200 python bench.py --workload c4 --no-cpu-baseline
step c4_off 200 env WB_TRIP_CMPBR=0 python bench.py --workload c4 --no-cpu-baseline
step c3k 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3 300 python bench.py --workload c3 --no-cpu-baseline
step mt 300 python bench.py --workload mt --no-cpu-baseline
step c4_on2 200 python bench.py --workload c4 --no-cpu-baseline
echo all done
