# r05 d: store write-back retention (wcal gap kernels) and VMM map costs per phase
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05d; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step vmm 120 $R/tools/ubench/vmm
step wcal 60 $R/tools/ubench/wcal
cd /tmp && export TMPDIR=/tmp
step wcal_write 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wcal_write -o run -- $R/tools/ubench/wcal
step wcal_fetch 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/wcal_fetch -o run -- $R/tools/ubench/wcal
echo all done
