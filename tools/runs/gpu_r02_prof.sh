# round-2 closing evidence: C2 bench line (with CPU baseline), rocprofv3 stats + PMC passes
set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 400 python bench.py > gpurun_out/prof/bench_c2.json 2> gpurun_out/prof/bench_c2.err || exit 1
bash tools/prof_bench.sh gpurun_out/prof/c2 --steps 3 --warmup 1 || exit 2
ls gpurun_out/prof/c2
