# r05 o: write-back of scattered 4-B stores against the L2 footprint (tools/ubench/alias.hip)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in 1024 256; do
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$w -o run -- $R/tools/ubench/alias 4096 4000 $w > $O/w$w.log 2>&1 || exit 1
  grep waves $O/w$w.log
done
echo done
