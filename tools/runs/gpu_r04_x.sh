# r04 x: the tail-call workload's closing profile and bench line after return_call moved
# into the compiled runs (same build as HEAD)
O=gpurun_out/r04x; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=150
step prof_tail 600 bash tools/prof_bench.sh gpurun_out/r04x/tail --workload tail --steps 3 --warmup 2
step prof_c1 900 bash tools/prof_bench.sh gpurun_out/r04x/c1 --workload c1 --steps 1 --warmup 1
