set -o pipefail
mkdir -p gpurun_out/g8
timeout -k 10 400 python -u tools/sched_stats.py > gpurun_out/g8/stats.txt 2>&1 || { cat gpurun_out/g8/stats.txt; exit 1; }
cat gpurun_out/g8/stats.txt
