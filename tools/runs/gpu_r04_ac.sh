# r04 ac: VALU-only group pre-test in the trip chain (WB_TRIP_PRE=n) -- parity with n = 4
# and C4 / C3 4K at n = 0 / 4 / 8
O=gpurun_out/r04ac; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 env WB_TRIP_PRE=4 python -u -m pytest tests/test_workloads.py tests/test_jit.py tests/test_depth_pick.py -m gpu -v --timeout 300 --timeout-method thread
for n in 0 4 8; do
  step c4_p$n 200 env WB_TRIP_PRE=$n python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
  step c3k_p$n 300 env WB_TRIP_PRE=$n python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
done
