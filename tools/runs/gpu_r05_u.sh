# r05 u: the leaf-call cache (return record + spills of a call whose callee makes no call,
# in VGPRs): call-heavy parity, C1 A/B (WB_LCC=0), fib anatomy, C2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05u; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-250)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_kat.py tests/test_jit.py tests/test_tailcall.py tests/test_depth_pick.py tests/test_deepstack.py tests/test_workloads.py -m gpu -v --timeout 300 --timeout-method thread
step c1 300 python bench.py --workload c1 --steps 2 --warmup 2 --no-cpu-baseline
step c1_off 300 env WB_LCC=0 python bench.py --workload c1 --steps 2 --warmup 2 --no-cpu-baseline
step fib 300 python tools/fib_probe.py
step c2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
step tail 300 python bench.py --workload tail --steps 3 --warmup 2 --no-cpu-baseline
echo all done
