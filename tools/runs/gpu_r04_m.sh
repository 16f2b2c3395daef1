# r04 m: the layout trial -- parity (layout / kat / workloads / growth / limits / hostcall)
# and the mt19937 + C3 benches with it (and with WB_GRANULE_TRIAL=0)
O=gpurun_out/r04m; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-220)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_layout.py tests/test_kat.py tests/test_workloads.py tests/test_memgrow.py tests/test_limits.py tests/test_hostcall.py tests/test_instance.py tests/test_memlimit.py -m gpu -v --timeout 200 --timeout-method thread
step mt 300 python bench.py --workload mt --steps 5 --warmup 2 --no-cpu-baseline
step mt_notrial 300 env WB_GRANULE_TRIAL=0 python bench.py --workload mt --steps 5 --warmup 2 --no-cpu-baseline
step c3 300 python bench.py --workload c3 --steps 2 --warmup 2 --no-cpu-baseline
