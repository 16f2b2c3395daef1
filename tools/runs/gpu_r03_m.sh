# r03: Lsched by distinct-pc enumeration (WB_LSCHED=1) against the DPP reductions:
# parity (partial waves on every engine, random modules), then C1/C4/C3 4K/C5 timings
O=gpurun_out/r03m; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 400 python -u -m pytest tests/test_workloads.py -m gpu -v --timeout 200 --timeout-method thread -k "partial_waves"
step rnd 300 env WB_LSCHED=1 python -u -m pytest tests/test_jit.py -m gpu -v --timeout 200 --timeout-method thread -k "random_modules"
for v in 1 0; do
  step c1_l$v 200 env WB_LSCHED=$v python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline
  step c4_l$v 200 env WB_LSCHED=$v python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline
  step c3_4k_l$v 200 env WB_LSCHED=$v python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
  step c5_l$v 200 env WB_LSCHED=$v python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --no-cpu-baseline
done
for f in $O/c*.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
