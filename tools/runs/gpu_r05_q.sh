# r05 q: br_table threading in trip mode (C4): parity (machine module, C4 at 64K, random
# modules), C4 bench A/B (WB_BRT_THREAD=0)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05q; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-250)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_tripcache.py tests/test_workloads.py tests/test_jit.py -m gpu -v --timeout 300 --timeout-method thread
step c4 300 python bench.py --workload c4 --steps 10 --warmup 5 --no-cpu-baseline
step c4_off 300 env WB_BRT_THREAD=0 python bench.py --workload c4 --steps 10 --warmup 5 --no-cpu-baseline
echo all done
