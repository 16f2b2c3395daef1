#!/bin/bash
# Per-config bench lines (BASELINE.json configs) on one GPU: writes $1/<workload>.json.
OUT=${1:-gpurun_out/bench_all}; mkdir -p $OUT
set -o pipefail
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $OUT/c2.json || exit 1
timeout -k 10 300 python bench.py --workload c1 --steps 2 --warmup 1 > $OUT/c1.json || exit 2
timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 > $OUT/c4.json || exit 3
timeout -k 10 300 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 > $OUT/c5.json || exit 4
timeout -k 10 300 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 > $OUT/c3_4k.json || exit 5
if [ "$FULL_C3" = 1 ]; then
  # configs[2] at full size: 64K instances x 1 MiB (262,144 i32) quicksort
  timeout -k 10 700 python bench.py --workload c3 --steps 1 --warmup 1 > $OUT/c3.json 2> $OUT/c3.log || exit 6
fi
echo done
