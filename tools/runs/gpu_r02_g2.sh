set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 300 python -u -m pytest tests/test_jit.py tests/test_simd.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/g2/tests.log 2>&1 || { tail -30 gpurun_out/g2/tests.log; exit 1; }
tail -1 gpurun_out/g2/tests.log
timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g2/c5_lds.json || exit 4
WB_VFRAME=1 timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g2/c5_vf.json || exit 5
cut -c1-200 gpurun_out/g2/c5_*.json
timeout -k 10 300 python -u tools/sched_stats.py > gpurun_out/g2/stats.txt 2>&1 || { cat gpurun_out/g2/stats.txt; exit 2; }
cat gpurun_out/g2/stats.txt
WB_VFRAME=1 timeout -k 10 300 python -u tools/sched_stats.py > gpurun_out/g2/stats_vf.txt 2>&1 || exit 3
grep -A3 c5-256k gpurun_out/g2/stats_vf.txt
