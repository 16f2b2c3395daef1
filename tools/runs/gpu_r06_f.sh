# r06 f: trip-chain function guards (WB_TRIP_GUARD) and the one-branch trip tail: parity of
# the trip-mode tests, then A/B on C3 4K, C4, C3 full
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06f; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step trips 600 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_jit.py -m gpu -v --timeout 300 --timeout-method thread
step c3k_g1 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3k_g0 200 env WB_TRIP_GUARD=0 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c4_g1 200 python bench.py --workload c4 --no-cpu-baseline
step c3_g1 300 python bench.py --workload c3 --no-cpu-baseline
step c3_g0 300 env WB_TRIP_GUARD=0 python bench.py --workload c3 --no-cpu-baseline
echo all done
