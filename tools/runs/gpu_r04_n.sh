# r04 n: return_call in the threaded core -- tail-call / JIT / scalar parity and the tail
# workload with the core's handler on and off (WB_TC_TAIL=0)
O=gpurun_out/r04o; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-220)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_tailcall.py tests/test_tables.py tests/test_apitest.py tests/test_workloads.py tests/test_jit.py tests/test_scalar.py tests/test_depth_pick.py tests/test_kat.py -m gpu -v --timeout 200 --timeout-method thread
step tail 300 python bench.py --workload tail --steps 5 --warmup 2
step tail_off 300 env WB_TC_TAIL=0 python bench.py --workload tail --steps 5 --warmup 2 --no-cpu-baseline
step c1 300 python bench.py --workload c1 --steps 3 --warmup 1 --no-cpu-baseline
step c3 300 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
step c4 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
