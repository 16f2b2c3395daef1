# r03 evidence at the start of the round: every config's rocprofv3 passes (HEAD code)
set -o pipefail
O=gpurun_out/r03b
mkdir -p $O
bash tools/prof_bench.sh $O/c2 || exit 1
bash tools/prof_bench.sh $O/c1 --workload c1 --steps 2 --warmup 1 || exit 2
bash tools/prof_bench.sh $O/c4 --workload c4 --steps 3 --warmup 1 || exit 3
bash tools/prof_bench.sh $O/c5 --workload c5 --instances 262144 --steps 3 --warmup 1 || exit 4
PROF_TIMEOUT=400 bash tools/prof_bench.sh $O/c3 --workload c3 --steps 1 --warmup 0 || exit 5
echo all done
