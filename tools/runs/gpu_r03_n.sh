# r03: scan loops unrolled inside the trips (WB_TRIP_SCAN, default 4) and forward chaining
# (WB_TRIP_CHAIN) -- trip-mode parity, C3 4K A/B, C1/C4 with trips forced, then C3 at
# 64K x 1 MiB with its CPU baseline
O=gpurun_out/r03n; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 500 python -u -m pytest tests/test_workloads.py tests/test_jit.py -m gpu -v --timeout 200 --timeout-method thread -k "partial_waves or scheduler_policies or random_modules or c3 or qsort"
step c3_4k 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
step c3_4k_s0 200 env WB_TRIP_SCAN=0 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
step c3_4k_c0 200 env WB_TRIP_CHAIN=0 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
step c3_4k_s0c0 200 env WB_TRIP_SCAN=0 WB_TRIP_CHAIN=0 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
step c1_trip 200 env WB_TRIP=1 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline
step c4_trip 200 env WB_TRIP=1 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline
step c3 600 python bench.py --workload c3 --steps 3 --warmup 1
for f in $O/c*.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
