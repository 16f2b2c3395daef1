# r05 c5: C5 repeated and fresh inputs with the argument buffers reused across SetArgs
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05c5; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step api 300 python -u -m pytest tests/test_apitest.py tests/test_instance.py tests/test_externref.py -m gpu -q --timeout 120 --timeout-method thread
step c5a 300 python bench.py --workload c5 --steps 5 --warmup 2
step c5b 300 python bench.py --workload c5 --steps 5 --warmup 2
echo all done
