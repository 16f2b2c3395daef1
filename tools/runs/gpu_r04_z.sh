# r04 z: trip dispatch by bitmask -- trip-mode parity (workloads: C3 full-size sample, C4,
# partial waves on every engine; random modules with trips forced; layout; scan) and the
# C4 / C3 A/B against the per-run compare chain (WB_TRIP_DISPATCH=0)
O=gpurun_out/r04z; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_workloads.py tests/test_jit.py tests/test_layout.py tests/test_depth_pick.py tests/test_memgrow.py tests/test_metering.py -m gpu -v --timeout 300 --timeout-method thread
step c4 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
step c4_old 200 env WB_TRIP_DISPATCH=0 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
step c3k 300 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
step c3k_old 300 env WB_TRIP_DISPATCH=0 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
step c3 300 env WB_GRANULE_TRIAL=0 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline
step c3_old 300 env WB_GRANULE_TRIAL=0 WB_TRIP_DISPATCH=0 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline
