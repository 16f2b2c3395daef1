# round-2 closing evidence: every config's bench line (with its CPU baseline), full-size C3,
# the scheduler statistics build, and the GPU suite
set -o pipefail
mkdir -p gpurun_out/final
FULL_C3=1 bash tools/bench_all.sh gpurun_out/final || exit 1
timeout -k 10 400 python -u tools/sched_stats.py > gpurun_out/final/sched_stats.txt 2>&1 || exit 2
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/tests.log 2>&1 || { tail -30 gpurun_out/final/tests.log; exit 3; }
tail -1 gpurun_out/final/tests.log
for f in gpurun_out/final/*.json; do echo $f; cut -c1-120 $f | sed 's/.*"value"/value/'; done
