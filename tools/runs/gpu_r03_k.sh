# r03: NaN payload liveness -- payload-exact GPU tests (new module, scalar and SIMD matrices)
# with the analysis, then C5 with it on and off, C2 unchanged.
O=gpurun_out/r03k; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 500 python -u -m pytest tests/test_nanobs.py tests/test_scalar.py tests/test_simd.py tests/test_workloads.py -m gpu -v --timeout 200 --timeout-method thread -k "nan or scalar or simd or c5 or mandel or partial"
step c5 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --cpu-seconds 4
step c5_off 200 env WB_NANOBS=0 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --no-cpu-baseline
step c2 200 python bench.py --no-cpu-baseline
