set -o pipefail
mkdir -p gpurun_out/g9
timeout -k 10 400 python -u -m pytest tests/test_scalar.py tests/test_simd.py tests/test_jit.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g9/t1.log 2>&1 || { tail -30 gpurun_out/g9/t1.log; exit 1; }
tail -1 gpurun_out/g9/t1.log
timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g9/c5.json || exit 2
cut -c1-150 gpurun_out/g9/c5.json | sed 's/.*"value"/value/'
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g9/tests.log 2>&1 || { tail -30 gpurun_out/g9/tests.log; exit 3; }
tail -1 gpurun_out/g9/tests.log
