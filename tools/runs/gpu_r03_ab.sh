# r03: constant-address stores in the forwarding copy (C2's loop loses its 48 address
# instructions per compression) and the opt-in compare-mask branch for C5 -- parity, then
# C2 and C5 A/Bs
O=gpurun_out/r03ab; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 700 env WB_CST_STORE=1 python -u -m pytest tests/test_forward.py tests/test_inline.py tests/test_workloads.py tests/test_kat.py tests/test_jit.py -m gpu -v --timeout 200 --timeout-method thread
step tests_cmpany 400 env WB_CMPANY=1 python -u -m pytest tests/test_fold.py tests/test_simd.py tests/test_nanobs.py tests/test_workloads.py -k "fold or simd or nanobs or c5 or mandel" -m gpu -v --timeout 200 --timeout-method thread
step c2 200 env WB_CST_STORE=1 python bench.py
step c2_nocst 200 python bench.py --no-cpu-baseline
step c5_cmpany 200 env WB_CMPANY=1 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --cpu-seconds 4
step c5 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1 --no-cpu-baseline
for f in $O/c*.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.4g'%d['value'], '%.4f'%d['ms_per_step'])" 2>/dev/null); done
