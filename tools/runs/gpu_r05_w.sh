# r05 w: the host-mapped "parked" word (a Run with no lane parked skips the service round's
# status copy): every host-round test, then C5 / C2 / mt step times
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05w; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_hostcall.py tests/test_hostcost.py tests/test_wasi.py tests/test_deepstack.py tests/test_memgrow.py tests/test_tailcall.py tests/test_multidevice.py tests/test_metering.py -m gpu -v --timeout 300 --timeout-method thread
step c5 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline
step c2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
echo all done
