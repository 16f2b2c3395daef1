# r05 f: C3 write traffic by trip-mode feature (tools/c3_writes.py knob variants, 64K x 4K)
# WRITE_SIZE and FETCH_SIZE
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05f; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
timeout -k 10 60 $R/tools/ubench/vmm > $O/vmm.log 2>&1; rc=$?; echo "vmm rc=$rc $(tail -1 $O/vmm.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step plain 200 python3 $R/tools/c3_writes.py --only base,trip0,scan0,chain0,split0,hyb0
cd /tmp && export TMPDIR=/tmp
step write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/tools/c3_writes.py --only base,trip0,scan0,chain0,split0,hyb0
step fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/c3_writes.py --only base,trip0,scan0,chain0,split0,hyb0
echo all done
