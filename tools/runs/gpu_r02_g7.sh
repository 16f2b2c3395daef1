set -o pipefail
mkdir -p gpurun_out/g7
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g7/c2.json || exit 1
timeout -k 10 200 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g7/c1.json || exit 2
timeout -k 10 200 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g7/c4.json || exit 3
timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g7/c5.json || exit 4
timeout -k 10 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g7/c3_4k.json || exit 5
timeout -k 10 400 python bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/g7/c3_full.json || exit 6
for f in gpurun_out/g7/*.json; do echo $f; cut -c1-150 $f | sed 's/.*"value"/value/'; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g7/tests.log 2>&1 || { tail -30 gpurun_out/g7/tests.log; exit 7; }
tail -1 gpurun_out/g7/tests.log
