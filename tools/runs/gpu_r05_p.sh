# r05 p: C3 4K against the scan window (WB_TRIP_SCAN 2/3/4): is the trip bound by load requests?
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05p; mkdir -p $O
for s in 4 3 2; do
  timeout -k 10 300 env WB_TRIP_SCAN=$s python $R/bench.py --workload c3 --elements 4096 --steps 3 --warmup 3 --no-cpu-baseline > $O/s$s.log 2>&1 || exit 1
  echo "scan $s: $(grep -o '"value": [0-9.e+]*' $O/s$s.log)"
done
