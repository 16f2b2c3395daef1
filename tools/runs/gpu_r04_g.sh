# r04 g: fall-through layout of the compiled runs -- parity (JIT / fold / forward / tail /
# workloads / scalar / simd) and A/B benches on C1, C4, C5, C2
O=gpurun_out/r04h; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_jit.py tests/test_fold.py tests/test_forward.py tests/test_workloads.py tests/test_scalar.py tests/test_simd.py tests/test_depth_pick.py tests/test_nanobs.py tests/test_inline.py tests/test_metering.py -m gpu -v --timeout 200 --timeout-method thread
for w in c5 c4 c1 c2; do
  case $w in c5) a="--instances 262144 --steps 10 --warmup 2";; c1) a="--steps 3 --warmup 1";; c4) a="--steps 10 --warmup 2";; c2) a="";; esac
  step ${w}_layout 200 python bench.py --workload $w $a --no-cpu-baseline
  step ${w}_nolayout 200 env WB_LAYOUT=0 python bench.py --workload $w $a --no-cpu-baseline
done
