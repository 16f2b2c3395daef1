# r03 closing A: the whole -m gpu suite at HEAD, then every config's bench line with its
# CPU baseline, and two A/Bs (C1 pc-only picks; C3 4K SIMT-only with depth picks)
O=gpurun_out/r03t; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step c2 200 python bench.py
step c1 200 python bench.py --workload c1 --steps 3 --warmup 1
step c4 200 python bench.py --workload c4 --steps 3 --warmup 1
step c5 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1
step mt 200 python bench.py --workload mt --steps 2 --warmup 1
step c3_4k 200 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 1
step c3_4k_simt 200 env WB_TRIP=0 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
step c1_pc 200 env WB_DEPTH=0 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline
step c3 300 python bench.py --workload c3 --steps 3 --warmup 1
for f in $O/c*.log $O/mt.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
