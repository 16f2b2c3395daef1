# r06 zu: the trips' exit threshold (WB_TRIP_OUTSH=k: leave when outside > 2^k x inside) on C4, C3 4K
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zu; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 300 python -u -m pytest tests/test_workloads.py -k "collatz or c4" -m gpu -v --timeout 200 --timeout-method thread
step c4_0 200 python bench.py --workload c4 --no-cpu-baseline
step c4_1 200 env WB_TRIP_OUTSH=1 python bench.py --workload c4 --no-cpu-baseline
step c4_2 200 env WB_TRIP_OUTSH=2 python bench.py --workload c4 --no-cpu-baseline
step c4_3 200 env WB_TRIP_OUTSH=3 python bench.py --workload c4 --no-cpu-baseline
step c3k_0 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3k_2 200 env WB_TRIP_OUTSH=2 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
echo all done
