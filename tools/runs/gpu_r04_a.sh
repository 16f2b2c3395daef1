# r04 a: paged memory growth (default page limit 65536, device pool) -- its tests, the
# memory-limit / workload / host-call parity tests, then the default bench line
O=gpurun_out/r04a; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step grow 400 python -u -m pytest tests/test_memgrow.py tests/test_memlimit.py -m gpu -v --timeout 200 --timeout-method thread
step parity 600 python -u -m pytest tests/test_workloads.py tests/test_hostcall.py tests/test_wasi.py tests/test_bulk.py tests/test_instance.py -m gpu -v --timeout 200 --timeout-method thread
step c2 200 python bench.py
