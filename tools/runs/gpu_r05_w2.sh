# r05 w2: 16-byte scan-window loads (WB_TRIP_WIDE): trip parity tests, then C3 A/B
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05w2; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step trip 400 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py -m gpu -v --timeout 200 --timeout-method thread
step c3_wide 300 python bench.py --workload c3
step c3_base 300 env WB_TRIP_WIDE=0 python bench.py --workload c3
step c3_wide2 300 python bench.py --workload c3
echo all done
