# r04 e: LPT order sorted on the device -- C5 A/B, parity, C1/C4/C2 lines
O=gpurun_out/r04e; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step c5_lpt 200 python bench.py --workload c5 --instances 262144 --steps 10 --warmup 2 --no-cpu-baseline
WB_LPT=0 step c5_nolpt 200 python bench.py --workload c5 --instances 262144 --steps 10 --warmup 2 --no-cpu-baseline
step tests 400 python -u -m pytest tests/test_workloads.py -m gpu -v --timeout 200 --timeout-method thread -k "c5 or partial or mandel"
step c1 200 python bench.py --workload c1 --steps 3 --warmup 1 --no-cpu-baseline
step c4 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
step c2 200 python bench.py --no-cpu-baseline
