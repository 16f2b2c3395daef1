# r03: known-site return tests (a return whose lanes all hold one of its function's first
# two call-site records goes straight there), RET without a second stack check after its
# run's POST_CALL -- parity incl. the recursion matrix, then C1 / C5 / C2 and the fib probe
O=gpurun_out/r03w; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 700 python -u -m pytest tests/test_depth_pick.py tests/test_kat.py tests/test_tailcall.py tests/test_scalar.py tests/test_workloads.py tests/test_jit.py tests/test_big_frames.py tests/test_apitest.py tests/test_hostcall.py tests/test_metering.py tests/test_inline.py tests/test_forward.py -m gpu -v --timeout 200 --timeout-method thread
step probe 300 python tools/fib_probe.py
step c1 200 python bench.py --workload c1 --steps 3 --warmup 1 --cpu-seconds 4
step c5 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --no-cpu-baseline
step mt 200 python bench.py --workload mt --steps 2 --warmup 1 --no-cpu-baseline
step c2 200 python bench.py --no-cpu-baseline
cat $O/probe.log
for f in $O/c*.log $O/mt.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
