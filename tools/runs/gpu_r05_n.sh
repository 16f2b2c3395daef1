# r05 n: L2 set aliasing between waves (tools/ubench/alias.hip): time and WRITE_SIZE per stride
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05n; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/ubench/alias 4096 4000 > $O/plain.log 2>&1 && cat $O/plain.log &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $R/tools/ubench/alias 4096 4000 > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $R/tools/ubench/alias 4096 4000 > $O/write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $R/tools/ubench/alias 4096 4000 > $O/fetch.log 2>&1 &&
echo done
