# r03: trip mode first GPU check -- parity on the divergent workloads, then A/B timings
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_workloads.py -m gpu -x -v --timeout 120 --timeout-method thread -k "scheduler_policies and (trip or notrip)" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -3 $O/t1.log
timeout -k 10 300 python -u -m pytest tests/test_jit.py -m gpu -x -v --timeout 120 --timeout-method thread -k "random_modules and trip" > $O/t2.log 2>&1 || { tail -40 $O/t2.log; exit 2; }
tail -3 $O/t2.log
for t in 0 1; do
  WB_TRIP=$t timeout -k 10 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --cpu-seconds 4 > $O/c3_4k_t$t.json 2> $O/c3_4k_t$t.err || { tail $O/c3_4k_t$t.err; exit 3; }
  WB_TRIP=$t timeout -k 10 200 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_t$t.json 2> $O/c4_t$t.err || { tail $O/c4_t$t.err; exit 4; }
  WB_TRIP=$t timeout -k 10 200 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline > $O/c1_t$t.json 2> $O/c1_t$t.err || { tail $O/c1_t$t.err; exit 5; }
  WB_TRIP=$t timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_t$t.json 2> $O/c5_t$t.err || { tail $O/c5_t$t.err; exit 6; }
done
for f in $O/*.json; do echo $f $(python3 -c "import json;d=json.load(open('$f'));print('%.3g'%d['value'], '%.2f'%d['ms_per_step'])"); done
