# r03: an f64x2 compare feeding a fused any_true branch leaves the lane masks for the
# branch (C5's escape test: 12 VALU instead of 16) -- parity, then C5 with and without
O=gpurun_out/r03aa; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 700 env WB_CMPANY=1 python -u -m pytest tests/test_fold.py tests/test_simd.py tests/test_nanobs.py tests/test_workloads.py tests/test_jit.py -m gpu -v --timeout 200 --timeout-method thread
step c5 200 env WB_CMPANY=1 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --cpu-seconds 4
step c5_base 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --no-cpu-baseline
step c5_nofold 200 env WB_FOLD=0 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --no-cpu-baseline
for f in $O/c*.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
