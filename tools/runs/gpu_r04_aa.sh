# r04 aa: what the trip loop's per-run lane tests cost -- C4 and C3 4K with each stage-B
# test repeated 0 / 1 / 3 extra times (WB_TRIP_DUP, a measurement aid: the repeats only run
# when the run is absent)
O=gpurun_out/r04aa; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-160)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
for d in 0 1 3; do
  step c4_d$d 200 env WB_TRIP_DUP=$d python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline
  step c3k_d$d 300 env WB_TRIP_DUP=$d python bench.py --workload c3 --elements 4096 --steps 3 --warmup 2 --no-cpu-baseline
done
