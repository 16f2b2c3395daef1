set -o pipefail
mkdir -p gpurun_out/g3
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g3/c2.json || exit 1
timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g3/c5_lds.json || exit 4
WB_VFRAME=1 timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g3/c5_vf.json || exit 5
timeout -k 10 200 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g3/c1.json || exit 6
timeout -k 10 200 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g3/c4.json || exit 7
for f in gpurun_out/g3/*.json; do echo $f; cut -c1-150 $f | sed 's/.*"value"/value/'; done
timeout -k 10 400 python -u -m pytest tests/test_workloads.py tests/test_simd.py tests/test_scalar.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g3/tests.log 2>&1 || { tail -30 gpurun_out/g3/tests.log; exit 2; }
tail -1 gpurun_out/g3/tests.log
