# r03: trip mode picked for call-free modules whose lanes part ways inside loops (C4) --
# parity (random modules may now pick trips too; C4 at 64K with traps), C4 default bench
O=gpurun_out/r03p; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 500 python -u -m pytest tests/test_workloads.py tests/test_jit.py tests/test_scalar.py tests/test_metering.py -m gpu -v --timeout 200 --timeout-method thread
step c4 200 python bench.py --workload c4 --steps 5 --warmup 1 --cpu-seconds 4
step c1 200 python bench.py --workload c1 --steps 2 --warmup 1 --cpu-seconds 4
step c5 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --cpu-seconds 4
for f in $O/c*.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
