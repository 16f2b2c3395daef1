# r04 p: Reset deferred into the interpreter's prologue -- parity on every reset / memory /
# state consumer, then C5 / C4 / C2 / C1 with it and without (WB_DEFER_RESET=0)
O=gpurun_out/r04p; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 1000 python -u -m pytest tests/test_instance.py tests/test_hostcall.py tests/test_memgrow.py tests/test_workloads.py tests/test_memlimit.py tests/test_multidevice.py tests/test_metering.py tests/test_imports.py tests/test_abi.py tests/test_layout.py tests/test_tables.py tests/test_apitest.py tests/test_wasi.py tests/test_bulk.py -m gpu -v --timeout 200 --timeout-method thread
for w in c5 c4 c2; do
  case $w in c5) a="--instances 262144 --steps 10 --warmup 2";; c4) a="--steps 10 --warmup 2";; c2) a="";; esac
  step ${w} 200 python bench.py --workload $w $a --no-cpu-baseline
  step ${w}_nodefer 200 env WB_DEFER_RESET=0 python bench.py --workload $w $a --no-cpu-baseline
done
