# r03 re-entry: state at HEAD -- the whole -m gpu suite, then every bench config with
# trip mode on and off. A failing test (pytest rc 1) does not stop the script; anything
# else (a crash, a timeout) does.
O=gpurun_out/r03e; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $n"; exit $rc; fi
}
step gputests 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
for t in 1 0; do
  step c3_4k_t$t 200 env WB_TRIP=$t python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --cpu-seconds 4
  step c4_t$t 200 env WB_TRIP=$t python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline
  step c1_t$t 200 env WB_TRIP=$t python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline
  step c5_t$t 200 env WB_TRIP=$t python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline
done
step mt 200 python bench.py --workload mt --steps 3 --warmup 1 --cpu-seconds 4
step c2 200 python bench.py --no-cpu-baseline
for f in $O/c*.log $O/mt.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
