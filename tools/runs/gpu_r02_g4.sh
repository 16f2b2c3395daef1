set -o pipefail
mkdir -p gpurun_out/g4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/g4/smoke.log 2>&1 || { tail -20 gpurun_out/g4/smoke.log; exit 1; }
tail -1 gpurun_out/g4/smoke.log
timeout -k 10 200 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g4/c1.json || exit 2
timeout -k 10 200 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g4/c4.json || exit 3
WB_VFRAME=1 timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g4/c5_vf.json || exit 4
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g4/c2.json || exit 5
timeout -k 10 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g4/c3.json || exit 7
WB_SIMT=1 timeout -k 10 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g4/c3_simt.json || exit 8
for f in gpurun_out/g4/*.json; do echo $f; cut -c1-150 $f | sed 's/.*"value"/value/'; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g4/tests.log 2>&1 || { tail -30 gpurun_out/g4/tests.log; exit 6; }
tail -1 gpurun_out/g4/tests.log
