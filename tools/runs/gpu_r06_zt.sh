# r06 zt: trip mode forced (WB_TRIP=1) on the SIMT configs after the every-16th-trip convergence
# test: C5, C1, tail calls against their default (SIMT) runs
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zt; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step c5_trip 300 env WB_TRIP=1 python bench.py --workload c5 --no-cpu-baseline
step c1_trip 200 env WB_TRIP=1 python bench.py --workload c1 --no-cpu-baseline
step c2_trip 200 env WB_TRIP=1 python bench.py --no-cpu-baseline
echo all done
