# r05 p2: same-build profiles at HEAD for the headline line (C2) and C5
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05p; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=150
step prof_c2 600 bash $R/tools/prof_bench.sh gpurun_out/r05p/c2 --steps 5 --warmup 2
step prof_c5 600 bash $R/tools/prof_bench.sh gpurun_out/r05p/c5 --workload c5 --instances 262144 --steps 5 --warmup 2
echo all done
