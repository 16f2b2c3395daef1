# r05 c: counter calibration -- tools/ubench/wcal (known byte counts for streaming and
# scattered 4-byte stores in the interpreter's 128-byte-granule layout) under WRITE_SIZE /
# FETCH_SIZE / kernel trace, and the new coalesced hash kernel on C3 4K (trace + FETCH_SIZE)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05c; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
# (an API refusal exits 1 and is not fatal here; anything else stops the script)
timeout -k 10 60 $R/tools/ubench/vmm > $O/vmm.log 2>&1; rc=$?
echo "vmm rc=$rc $(tail -1 $O/vmm.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after vmm"; exit $rc; fi
step wcal 60 $R/tools/ubench/wcal
cd /tmp && export TMPDIR=/tmp
step wcal_trace 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wcal_trace -o run -- $R/tools/ubench/wcal
step wcal_write 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/wcal_write -o run -- $R/tools/ubench/wcal
step wcal_fetch 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/wcal_fetch -o run -- $R/tools/ubench/wcal
step hash_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hash_trace -o run -- python3 $R/bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
step hash_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/hash_fetch -o run -- python3 $R/bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
echo all done
