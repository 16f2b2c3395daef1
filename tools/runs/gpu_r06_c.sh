# r06 c: WASI fs mismatch diagnosis; batched trip lane tests (WB_TRIP_BATCH) -- parity of
# the trip-mode tests, then A/B on C4, C3 4K and C3 full
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06c; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step fsdiff 200 python -u tools/wasi_fs_diff.py
step trips 600 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py -m gpu -v --timeout 300 --timeout-method thread
step c4_b1 200 python bench.py --workload c4 --no-cpu-baseline
step c4_b0 200 env WB_TRIP_BATCH=0 python bench.py --workload c4 --no-cpu-baseline
step c3k_b1 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3k_b0 200 env WB_TRIP_BATCH=0 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3_b1 300 python bench.py --workload c3 --no-cpu-baseline
echo all done
