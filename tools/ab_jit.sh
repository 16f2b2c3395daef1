#!/bin/bash
# A/B of the compiled runs (WB_JIT=1 vs 0) on the BASELINE configs, no CPU baseline:
# writes $1/<workload>_jit<0|1>.json
OUT=${1:-gpurun_out/ab_jit}; mkdir -p $OUT
set -o pipefail
for j in 1 0; do
  WB_JIT=$j timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/c2_jit$j.json || exit 1
  WB_JIT=$j timeout -k 10 200 python bench.py --no-cpu-baseline --workload c1 --steps 2 --warmup 1 > $OUT/c1_jit$j.json || exit 2
  WB_JIT=$j timeout -k 10 200 python bench.py --no-cpu-baseline --workload c4 --steps 3 --warmup 1 > $OUT/c4_jit$j.json || exit 3
  WB_JIT=$j timeout -k 10 200 python bench.py --no-cpu-baseline --workload c3 --elements 4096 --steps 2 --warmup 1 > $OUT/c3_4k_jit$j.json || exit 4
done
for f in $OUT/*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('%-28s %.4g instr/s  %.3f ms/step' % ('$f'.split('/')[-1], d['value'], d['ms_per_step']))"; done
