# r05 j: the reserved layout grown in the grow service round (live copy) and at Reset;
# memgrow / hostcall / layout tests, C3 vs growing C3 at 4K and 1 MiB
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05j; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_deepstack.py tests/test_hostcall.py tests/test_hostcost.py -m gpu -v --timeout 300 --timeout-method thread
step c3gk 300 python bench.py --workload c3grow --elements 4096 --steps 3 --warmup 3 --no-cpu-baseline
step c3g 600 python bench.py --workload c3grow --steps 2 --warmup 3 --no-cpu-baseline
echo all done
