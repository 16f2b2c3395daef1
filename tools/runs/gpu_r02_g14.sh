set -o pipefail
mkdir -p gpurun_out/g14
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/g14/c2.json || exit 1
WB_INLINE=0 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/g14/c2_noinl.json || exit 2
for f in gpurun_out/g14/*.json; do echo $f; cut -c1-200 $f | sed 's/.*"value"/value/'; done
timeout -k 10 400 python -u -m pytest tests/test_workloads.py tests/test_kat.py tests/test_jit.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g14/tests.log 2>&1 || { tail -30 gpurun_out/g14/tests.log; exit 3; }
tail -1 gpurun_out/g14/tests.log
