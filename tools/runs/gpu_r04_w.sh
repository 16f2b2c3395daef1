# r04 w: return_call compiled into the JIT runs -- tail-call / JIT / recursion parity and the
# tail, C1 and C2 benches
O=gpurun_out/r04w; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_tailcall.py tests/test_jit.py tests/test_depth_pick.py tests/test_scalar.py tests/test_kat.py tests/test_workloads.py -m gpu -v --timeout 300 --timeout-method thread
step tail 300 python bench.py --workload tail --steps 5 --warmup 2 --no-cpu-baseline
step c1 300 python bench.py --workload c1 --steps 3 --warmup 1 --no-cpu-baseline
step c2 300 python bench.py --no-cpu-baseline
