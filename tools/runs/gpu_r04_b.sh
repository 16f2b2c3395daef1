# r04 b: multi-device contexts, host tail calls, build hash, then the whole -m gpu suite
O=gpurun_out/r04b; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step new 400 python -u -m pytest tests/test_multidevice.py tests/test_tailcall.py tests/test_abi.py -m gpu -v --timeout 200 --timeout-method thread
step all 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
