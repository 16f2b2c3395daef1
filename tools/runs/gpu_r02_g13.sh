set -o pipefail
mkdir -p gpurun_out/g13
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/g13/c2.json || exit 1
cut -c1-200 gpurun_out/g13/c2.json
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g13/tests.log 2>&1 || { tail -30 gpurun_out/g13/tests.log; exit 2; }
tail -1 gpurun_out/g13/tests.log
