# r06 r: same-build rocprofv3 profiles at HEAD (all passes of tools/prof_bench.sh): C2, C5, C4
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06r; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=150
step prof_c2 400 bash $R/tools/prof_bench.sh gpurun_out/r06r/c2 --steps 5 --warmup 2
step prof_c5 400 bash $R/tools/prof_bench.sh gpurun_out/r06r/c5 --workload c5 --steps 3 --warmup 1
step prof_c4 400 bash $R/tools/prof_bench.sh gpurun_out/r06r/c4 --workload c4
echo all done
