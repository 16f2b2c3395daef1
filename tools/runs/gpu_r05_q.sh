# r05 q: same-build profiles at HEAD (after the fused reset) for C2, C5, C4, C1, C3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05q; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-120)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=150
step prof_c2 600 bash $R/tools/prof_bench.sh gpurun_out/r05q/c2 --steps 5 --warmup 2
step prof_c5 600 bash $R/tools/prof_bench.sh gpurun_out/r05q/c5 --workload c5 --instances 262144 --steps 5 --warmup 2
step prof_c4 600 bash $R/tools/prof_bench.sh gpurun_out/r05q/c4 --workload c4 --steps 5 --warmup 2
step prof_c1 900 bash $R/tools/prof_bench.sh gpurun_out/r05q/c1 --workload c1 --steps 1 --warmup 1
export PROF_TIMEOUT=240
step prof_c3 1200 bash $R/tools/prof_bench.sh gpurun_out/r05q/c3 --workload c3 --steps 1 --warmup 3
echo all done
