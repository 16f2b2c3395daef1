set -o pipefail
mkdir -p gpurun_out/g15
timeout -k 10 300 python -u -m pytest tests/test_inline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g15/t1.log 2>&1 || { tail -30 gpurun_out/g15/t1.log; exit 1; }
tail -1 gpurun_out/g15/t1.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/g15/c2.json || exit 2
cut -c1-200 gpurun_out/g15/c2.json
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g15/tests.log 2>&1 || { tail -30 gpurun_out/g15/tests.log; exit 3; }
tail -1 gpurun_out/g15/tests.log
