set -o pipefail
mkdir -p gpurun_out/g6
timeout -k 10 60 python -u tools/simt_probe.py 64 > gpurun_out/g6/probe.log 2>&1 || { tail -5 gpurun_out/g6/probe.log; exit 1; }
grep "bad lanes" gpurun_out/g6/probe.log
timeout -k 10 200 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g6/c1.json || exit 2
timeout -k 10 200 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g6/c4.json || exit 3
WB_VFRAME=1 timeout -k 10 200 python bench.py --workload c5 --instances 262144 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g6/c5_vf.json || exit 4
WB_SIMT=1 timeout -k 10 200 python bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g6/c3_simt.json || exit 5
for f in gpurun_out/g6/*.json; do echo $f; cut -c1-150 $f | sed 's/.*"value"/value/'; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g6/tests.log 2>&1 || { tail -30 gpurun_out/g6/tests.log; exit 6; }
tail -1 gpurun_out/g6/tests.log
