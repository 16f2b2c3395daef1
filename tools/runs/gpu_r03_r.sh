# r03: fast transfers (one branch for the common case), RET stack check folded into the
# record, one call-stack check per POST_CALL..CALL run -- parity, then C1 / C4 / C3 4K / C5 / C2
O=gpurun_out/r03r; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_scalar.py tests/test_workloads.py tests/test_jit.py tests/test_kat.py tests/test_tailcall.py tests/test_inline.py tests/test_forward.py tests/test_big_frames.py tests/test_metering.py -m gpu -v --timeout 200 --timeout-method thread
step c1 200 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline
step c4 200 python bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline
step c3_4k 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
step c5 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --no-cpu-baseline
step mt 200 python bench.py --workload mt --steps 2 --warmup 1 --no-cpu-baseline
step c2 200 python bench.py --no-cpu-baseline
for f in $O/c*.log $O/mt.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
