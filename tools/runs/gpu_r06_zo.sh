# r06 zo: the convergence test's period (WB_TRIP_CONVP=k: every 2^k-th trip) on C4 and C3 4K
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zo; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
for k in 1 2 3 4 6; do
  step c4_p$k 200 env WB_TRIP_CONVP=$k python bench.py --workload c4 --no-cpu-baseline
done
for k in 2 4; do
  step c3k_p$k 200 env WB_TRIP_CONVP=$k python bench.py --workload c3 --elements 4096 --no-cpu-baseline
done
step mt_p4 300 env WB_TRIP_CONVP=4 python bench.py --workload mt --no-cpu-baseline
echo all done
