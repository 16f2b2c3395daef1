# r04 j: fused reset kernel, parallel wave-order scan, event sync -- parity on the reset /
# instance / host-call / growth / workload tests, then C5/C4/C2/C1 benches and a C5 trace
O=gpurun_out/r04k; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_instance.py tests/test_hostcall.py tests/test_memgrow.py tests/test_workloads.py tests/test_memlimit.py tests/test_multidevice.py tests/test_metering.py tests/test_imports.py tests/test_abi.py tests/test_kat.py -m gpu -v --timeout 200 --timeout-method thread
step c5 200 python bench.py --workload c5 --instances 262144 --steps 10 --warmup 2 --no-cpu-baseline
step c4 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
step c2 200 python bench.py --workload c2 --no-cpu-baseline
step c3 300 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step c5trace 300 rocprofv3 --kernel-trace --output-format csv -d $O/c5t -o run -- python3 bench.py --workload c5 --instances 262144 --steps 10 --warmup 2 --no-cpu-baseline
