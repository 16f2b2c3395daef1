# r06 x: branch-free scan stage B (WB_TRIP_SCANBF), 16-byte scan windows (WB_TRIP_X4) on top of
# the load-cache stage without re-checks: trip-mode and JIT parity, then A/B on C3 4K, C3 1 MiB
# and C3 on memory 1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06x; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 700 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_xmem_jit.py tests/test_jit.py -m gpu -v --timeout 300 --timeout-method thread
step c3k_bf 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3k_nobf 200 env WB_TRIP_SCANBF=0 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3k_nox4 200 env WB_TRIP_X4=0 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3 300 python bench.py --workload c3 --no-cpu-baseline
step c3x 300 python bench.py --workload c3x --no-cpu-baseline
echo all done
