#!/bin/bash
# A/B of the wave scheduler (WB_SCHED=0 min pc, 1 largest group) on the divergent configs.
OUT=${1:-gpurun_out/ab_sched}; mkdir -p $OUT
set -o pipefail
for s in ${SCHEDS:-0 1}; do
  WB_SCHED=$s timeout -k 10 300 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c1_s$s.json || exit 1
  WB_SCHED=$s timeout -k 10 300 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c3_s$s.json || exit 2
  WB_SCHED=$s timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c4_s$s.json || exit 3
  WB_SCHED=$s timeout -k 10 300 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5_s$s.json || exit 4
  WB_SCHED=$s timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c2_s$s.json || exit 5
done
echo done
