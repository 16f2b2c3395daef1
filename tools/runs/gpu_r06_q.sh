# r06 q: threaded-core handlers for XLD / XST (V blob): the extra-memory tests (core-only
# variants run the handlers alone); then C5 / mt fresh inputs with WB_ORDER_ANY=1 against
# the default, and C1 after the pc-0 re-aim trim
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06q; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step xtests 600 python -u -m pytest tests/test_xmem_jit.py tests/test_multimem.py tests/test_tripcache.py -m gpu -v --timeout 300 --timeout-method thread
step c3xk_core 300 env WB_JIT=0 python bench.py --workload c3x --elements 4096 --no-cpu-baseline
step c3k_core 300 env WB_JIT=0 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c5_def 300 python bench.py --workload c5 --no-cpu-baseline
step c5_any 300 env WB_ORDER_ANY=1 python bench.py --workload c5 --no-cpu-baseline
step mt_any 300 env WB_ORDER_ANY=1 python bench.py --workload mt --no-cpu-baseline
step c1 300 python bench.py --workload c1 --no-cpu-baseline
echo all done
