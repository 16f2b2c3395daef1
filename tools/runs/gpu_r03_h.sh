# r03: hybrid trip/SIMT scheduling -- the trip-mode parity tests, C3 4K and mt19937 A/B
# (hybrid against trips alone), then C3 at 64K x 1 MiB: parity test, bench line with its
# CPU baseline, rocprofv3 passes of one step.
O=gpurun_out/r03h; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step triptests 500 python -u -m pytest tests/test_workloads.py tests/test_jit.py tests/test_kat.py -m gpu -v --timeout 200 --timeout-method thread -k "partial_waves or scheduler_policies or random_modules or c3 or mt19937 or qsort"
step c3_4k 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --cpu-seconds 4
step c3_4k_nohyb 200 env WB_HYBRID=0 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
step mt 200 python bench.py --workload mt --steps 3 --warmup 1 --cpu-seconds 4
step mt_g4 200 env WB_GRANULE=4 python bench.py --workload mt --steps 3 --warmup 1 --no-cpu-baseline
step c3 600 python bench.py --workload c3 --steps 3 --warmup 1
export PROF_TIMEOUT=240
step prof 1100 bash tools/prof_bench.sh gpurun_out/r03h/prof --workload c3 --steps 1 --warmup 0
