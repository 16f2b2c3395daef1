# r05 l: the successor-window prefetch (C3's j-scan in the same trip as the i-scan):
# parity (trip shortcuts module, workloads), C3 4K A/B (WB_TRIP_PF=0), C3 1 MiB
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05l; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_jit.py -m gpu -v --timeout 300 --timeout-method thread
step c3k 300 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 3 --no-cpu-baseline
step c3k_nopf 300 env WB_TRIP_PF=0 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 3 --no-cpu-baseline
step c3 400 python bench.py --workload c3 --steps 2 --warmup 3 --no-cpu-baseline
echo all done
