# r06 m: byte-field br_table, leaner i64 immediates: the engine / numerics tests, then C4,
# mt19937, C2 and C5
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06m; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_jit.py tests/test_scalar.py tests/test_workloads.py tests/test_tripcache.py tests/test_kat.py tests/test_simd.py tests/test_xmem_jit.py -m gpu -v --timeout 300 --timeout-method thread
step c4 200 python bench.py --workload c4 --no-cpu-baseline
step mt 300 python bench.py --workload mt --no-cpu-baseline
step c2 200 python bench.py --no-cpu-baseline
step c5 300 python bench.py --workload c5 --no-cpu-baseline
echo all done
