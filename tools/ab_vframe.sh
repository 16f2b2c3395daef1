#!/bin/bash
# A/B of the threaded core with frames in VGPRs (default) vs in LDS (WB_VFRAME=0) over
# the BASELINE configs on one GPU: writes $1/{vf,lds}_<workload>.json. Tuning aid.
OUT=${1:-gpurun_out/ab}; mkdir -p $OUT
set -o pipefail
for mode in vf lds; do
  if [ $mode = lds ]; then export WB_VFRAME=0; else unset WB_VFRAME; fi
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${mode}_c2.json || exit 1
  timeout -k 10 200 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/${mode}_c1.json || exit 2
  timeout -k 10 200 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${mode}_c4.json || exit 3
  timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${mode}_c5.json || exit 4
  timeout -k 10 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/${mode}_c3.json || exit 5
done
echo done
