# r03: rocprofv3 passes for C5 (NaN payload liveness) and C2 at HEAD
O=gpurun_out/r03l; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=120
step prof_c5 400 bash tools/prof_bench.sh gpurun_out/r03l/c5 --workload c5 --instances 262144 --steps 5 --warmup 1
step prof_c2 400 bash tools/prof_bench.sh gpurun_out/r03l/c2
