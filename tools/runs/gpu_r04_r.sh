# r04 r: trip-mode scan window of 8 -- C3 parity (workloads incl. 64K x 1 MiB sample, jit
# random modules, trips) and C3 4K / full benches at windows 8 and 4
O=gpurun_out/r04r; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_workloads.py tests/test_jit.py tests/test_layout.py -m gpu -v --timeout 300 --timeout-method thread
step c3k8 300 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
step c3k4 300 env WB_TRIP_SCAN=4 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
step c3f8 300 env WB_GRANULE_TRIAL=0 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline
step c3f4 300 env WB_GRANULE_TRIAL=0 WB_TRIP_SCAN=4 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline
