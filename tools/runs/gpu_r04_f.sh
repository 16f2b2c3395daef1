# r04 f: many data / element segments, the C driver on the GPU, LPT with partial waves
O=gpurun_out/r04f; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step new 600 python -u -m pytest tests/test_limits.py tests/test_abi.py tests/test_tables.py tests/test_bulk.py tests/test_instance.py -m gpu -v --timeout 200 --timeout-method thread
