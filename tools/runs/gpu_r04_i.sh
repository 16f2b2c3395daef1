# r04 i: C5 / C4 step timeline (kernel + copy trace) to find the per-step host/launch gaps
O=gpurun_out/r04i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/c5 -o run -- python3 bench.py --workload c5 --instances 262144 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5.log 2>&1 || { echo c5 failed; tail -5 $O/c5.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/c4 -o run -- python3 bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/c4.log 2>&1 || { echo c4 failed; tail -5 $O/c4.log; exit 1; }
find $O -name "*.csv" | head; tail -1 $O/c5.log | cut -c1-150
