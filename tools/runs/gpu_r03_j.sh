# r03: rocprofv3 passes at HEAD for C1, C4, C5 (256K) and mt19937 (one step each), then
# the PC-sampling probe (gpu_r03_i.sh)
O=gpurun_out/r03j; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=120
step prof_c1 600 bash tools/prof_bench.sh gpurun_out/r03j/c1 --workload c1 --steps 1 --warmup 0
step prof_c4 400 bash tools/prof_bench.sh gpurun_out/r03j/c4 --workload c4 --steps 3 --warmup 1
step prof_c5 400 bash tools/prof_bench.sh gpurun_out/r03j/c5 --workload c5 --instances 262144 --steps 3 --warmup 1
step prof_mt 400 bash tools/prof_bench.sh gpurun_out/r03j/mt --workload mt --steps 1 --warmup 0
step pcs 400 bash tools/runs/gpu_r03_i.sh
