# r03 closing B: rocprofv3 passes at HEAD (kernel trace + stats, HBM bytes, issue counts,
# wave-cycle split, exec-mask efficiency, VMEM latency) for C1, C2, C4, C5 (256K), mt19937
O=gpurun_out/r03u; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=120
step prof_c1 400 bash tools/prof_bench.sh gpurun_out/r03u/c1 --workload c1 --steps 1 --warmup 0
step prof_c2 300 bash tools/prof_bench.sh gpurun_out/r03u/c2 --steps 5 --warmup 1
step prof_c4 300 bash tools/prof_bench.sh gpurun_out/r03u/c4 --workload c4 --steps 3 --warmup 1
step prof_c5 300 bash tools/prof_bench.sh gpurun_out/r03u/c5 --workload c5 --instances 262144 --steps 3 --warmup 1
step prof_mt 300 bash tools/prof_bench.sh gpurun_out/r03u/mt --workload mt --steps 1 --warmup 0
