# r04 ab: grouped trip lane tests (WB_TRIP_GROUP=1) -- trip-mode parity with them on, then
# C4 / C3 4K / C3 full A/B against the per-run chain, and the chain's cost (WB_TRIP_DUP)
O=gpurun_out/r04ab; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 env WB_TRIP_GROUP=1 python -u -m pytest tests/test_workloads.py tests/test_jit.py tests/test_layout.py tests/test_depth_pick.py tests/test_memgrow.py -m gpu -v --timeout 300 --timeout-method thread
step c4_g 200 env WB_TRIP_GROUP=1 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
step c4 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
step c4_dup1 200 env WB_TRIP_DUP=1 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
step c3k_g 300 env WB_TRIP_GROUP=1 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
step c3k 300 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
step c3k_dup1 300 env WB_TRIP_DUP=1 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
