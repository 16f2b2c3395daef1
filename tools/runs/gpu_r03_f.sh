# r03: does a second wave per SIMD come for free on the latency-bound configs? Each
# divergent config at 64K instances (1 wave per SIMD) and at 128K (2 per SIMD); ms per
# step that barely moves means the SIMDs idle half the time at 64K.
O=gpurun_out/r03f; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $n"; exit $rc; fi
}
for n in 65536 131072; do
  step c1_$n 200 python bench.py --workload c1 --instances $n --steps 2 --warmup 1 --no-cpu-baseline
  step c4_$n 200 python bench.py --workload c4 --instances $n --steps 3 --warmup 1 --no-cpu-baseline
  step c3_4k_$n 200 python bench.py --workload c3 --elements 4096 --instances $n --steps 2 --warmup 1 --no-cpu-baseline
  step c3_4k_notrip_$n 200 env WB_TRIP=0 python bench.py --workload c3 --elements 4096 --instances $n --steps 2 --warmup 1 --no-cpu-baseline
done
# half waves: the 64K batch as 2048 launch waves of 32 lanes
step c1_half 200 env WB_HALF=1 python bench.py --workload c1 --steps 2 --warmup 1 --cpu-seconds 3
step c4_half 200 env WB_HALF=1 python bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 3
step c3_4k_half 200 env WB_HALF=1 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --cpu-seconds 3
step c3_4k_half_notrip 200 env WB_HALF=1 WB_TRIP=0 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --cpu-seconds 3
step c2_half 200 env WB_HALF=1 python bench.py --cpu-seconds 3 --steps 5
for f in $O/c*.log; do echo $f $(grep -h '"metric"' $f | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3g'%d['value'], '%.3f'%d['ms_per_step'])" 2>/dev/null); done
