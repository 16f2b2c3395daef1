# r06 za: inline-constant branch transfers: engine parity, then C3 4K, C4, C1, C3 1 MiB
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06za; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 800 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_xmem_jit.py tests/test_jit.py tests/test_kat.py tests/test_scalar.py -m gpu -v --timeout 300 --timeout-method thread
step c3k 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c4 200 python bench.py --workload c4 --no-cpu-baseline
step c1 200 python bench.py --workload c1 --no-cpu-baseline
step c3 300 python bench.py --workload c3 --no-cpu-baseline
echo all done
