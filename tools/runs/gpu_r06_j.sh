# r06 j: extra memories in granules (128 B for data-dependent addresses); XLD / XST (memories past the first): parity on every engine, then C3 on
# memory 1 against C3 (4K and full size), and C2 for the kernel's register allocation
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06j; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step xtests 400 python -u -m pytest tests/test_xmem_jit.py tests/test_multimem.py tests/test_tripcache.py -m gpu -v --timeout 200 --timeout-method thread
step c3k 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3xk 200 python bench.py --workload c3x --elements 4096 --no-cpu-baseline
step c3x 400 python bench.py --workload c3x --no-cpu-baseline
step c3 400 python bench.py --workload c3 --no-cpu-baseline
echo all done
