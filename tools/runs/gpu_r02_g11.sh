set -o pipefail
mkdir -p gpurun_out/g11
timeout -k 10 400 python -u -m pytest tests/test_jit.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g11/t1.log 2>&1 || { tail -30 gpurun_out/g11/t1.log; exit 1; }
tail -1 gpurun_out/g11/t1.log
timeout -k 10 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g11/c3_4k.json || exit 2
WB_SCAN=0 timeout -k 10 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g11/c3_4k_noscan.json || exit 3
for f in gpurun_out/g11/*.json; do echo $f; cut -c1-150 $f | sed 's/.*"value"/value/'; done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g11/tests.log 2>&1 || { tail -30 gpurun_out/g11/tests.log; exit 6; }
tail -1 gpurun_out/g11/tests.log
timeout -k 10 300 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/g11/c3_full.json || exit 7
cut -c1-150 gpurun_out/g11/c3_full.json
