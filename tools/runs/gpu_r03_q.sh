# r03: in-place lane-wise SIMD results -- SIMD / NaN / workload parity, C5 timing
O=gpurun_out/r03q; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 500 python -u -m pytest tests/test_simd.py tests/test_nanobs.py tests/test_workloads.py tests/test_jit.py tests/test_kat.py -m gpu -v --timeout 200 --timeout-method thread -k "simd or nan or mandel or c5 or workload_parity or random or mt19937 or partial"
step c5 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --cpu-seconds 4
step mt 200 python bench.py --workload mt --steps 3 --warmup 1 --no-cpu-baseline
for f in $O/c*.log $O/mt.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
