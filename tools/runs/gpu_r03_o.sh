# r03: the full -m gpu suite at HEAD, then trips forced on C5 and C2 (which rule picks trips)
O=gpurun_out/r03o; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $n"; exit $rc; fi
}
step gputests 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step c5_trip 200 env WB_TRIP=1 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --no-cpu-baseline
step c5 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --no-cpu-baseline
step c2_trip 200 env WB_TRIP=1 python bench.py --no-cpu-baseline --steps 10
step c4_trip_lsched 200 env WB_TRIP=1 WB_LSCHED=1 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline
for f in $O/c*.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
