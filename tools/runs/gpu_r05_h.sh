# r05 h: debug of the virtual-memory grow path (tools/vmm_debug.py), then the memgrow tests
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05h; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step dbg64 120 env WB_VMM_DEBUG=1 python3 tools/vmm_debug.py 64

echo all done
