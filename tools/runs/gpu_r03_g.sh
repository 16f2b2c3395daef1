# r03: C3 at its configs[2] size (64K x 1 MiB) with trip mode: the full-size parity test,
# the bench line with its CPU baseline, then the rocprofv3 passes of one step.
O=gpurun_out/r03g; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step c3test 400 python -u -m pytest tests/test_workloads.py -m gpu -v --timeout 380 --timeout-method thread -k "c3_64k_x_1mib"
step c3 600 python bench.py --workload c3 --steps 3 --warmup 1
export PROF_TIMEOUT=240
step prof 1500 bash tools/prof_bench.sh gpurun_out/r03g/prof --workload c3 --steps 1 --warmup 0
# mt19937 (not a config): SIMT + word interleave against the default (trip mode, 128-byte
# granules: its addresses depend on loaded data, so the static analysis calls it divergent)
step mt_t0_g4 200 env WB_TRIP=0 WB_GRANULE=4 python bench.py --workload mt --steps 3 --warmup 1 --no-cpu-baseline
step mt_t0 200 env WB_TRIP=0 python bench.py --workload mt --steps 3 --warmup 1 --no-cpu-baseline
