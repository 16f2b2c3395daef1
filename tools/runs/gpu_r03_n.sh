# r03: scan loops unrolled inside the trips (WB_TRIP_SCAN, default 4) -- trip-mode parity,
# C3 4K A/B, then C3 at 64K x 1 MiB with its CPU baseline
O=gpurun_out/r03n; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 500 python -u -m pytest tests/test_workloads.py tests/test_jit.py -m gpu -v --timeout 200 --timeout-method thread -k "partial_waves or scheduler_policies or random_modules or c3 or qsort"
for v in 4 2 0; do
  step c3_4k_s$v 200 env WB_TRIP_SCAN=$v python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
done
step c3 600 python bench.py --workload c3 --steps 3 --warmup 1
for f in $O/c*.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
