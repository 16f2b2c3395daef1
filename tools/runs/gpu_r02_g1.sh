set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/g1/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/g1/tests.log; exit 1; }
tail -2 gpurun_out/g1/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g1/smoke.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g1/c2.json || exit 3
timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g1/c5_lds.json || exit 4
WB_VFRAME=1 timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g1/c5_vf.json || exit 5
cat gpurun_out/g1/*.json | cut -c1-300
