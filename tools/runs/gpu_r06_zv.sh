# r06 zv: the exit threshold, larger k (WB_TRIP_OUTSH) on C4; mt, C3 4K at k = 6
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zv; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step c4_3 200 env WB_TRIP_OUTSH=3 python bench.py --workload c4 --no-cpu-baseline
step c4_4 200 env WB_TRIP_OUTSH=4 python bench.py --workload c4 --no-cpu-baseline
step c4_6 200 env WB_TRIP_OUTSH=6 python bench.py --workload c4 --no-cpu-baseline
step c3k_6 200 env WB_TRIP_OUTSH=6 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step mt_6 300 env WB_TRIP_OUTSH=6 python bench.py --workload mt --no-cpu-baseline
echo all done
