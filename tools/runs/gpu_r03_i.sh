# r03: can rocprofv3 PC-sample the compiled runs? List the PC-sampling configurations, then
# sample a short C1 run (8K instances, one step) by cycles.
O=gpurun_out/r03i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 60 rocprofv3 -L > $R/$O/list.log 2>&1; echo "list rc=$?"
grep -i -B2 -A12 "pc.sampl\|pc_sampl" $R/$O/list.log | head -60
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 --output-format csv -d $R/$O/pcs -o run -- python3 $R/bench.py --workload c1 --instances 8192 --steps 1 --warmup 0 --no-cpu-baseline > $R/$O/pcs.log 2>&1
echo "pcs rc=$?"; tail -5 $R/$O/pcs.log; ls -la $R/$O/pcs 2>/dev/null | head
