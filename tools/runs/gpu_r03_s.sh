# r03: depth-keyed SIMT picks for recursive modules -- parity, the fib anatomy probe with
# and without, C1 / C3 4K / C5 benches
O=gpurun_out/r03s; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_kat.py tests/test_tailcall.py tests/test_scalar.py tests/test_workloads.py tests/test_jit.py tests/test_big_frames.py tests/test_apitest.py tests/test_hostcall.py tests/test_metering.py -m gpu -v --timeout 200 --timeout-method thread
step probe 300 python tools/fib_probe.py
step probe_pc 300 env WB_DEPTH=0 python tools/fib_probe.py
step c1 200 python bench.py --workload c1 --steps 2 --warmup 1 --cpu-seconds 4
step c3_4k 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
cat $O/probe.log $O/probe_pc.log
for f in $O/c*.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
