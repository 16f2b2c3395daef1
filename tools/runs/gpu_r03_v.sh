# r03 closing C: rocprofv3 passes at HEAD for C3 at its configs[2] size (64K x 1 MiB)
O=gpurun_out/r03v; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=150
step prof_c3 1100 bash tools/prof_bench.sh gpurun_out/r03v/c3 --workload c3 --steps 1 --warmup 0
# the C2 trace pass again (its kernel time under the profiler against the bench step)
PROF_PASSES="trace" step prof_c2_trace 200 bash tools/prof_bench.sh gpurun_out/r03v/c2 --steps 20 --warmup 2
