# r06 d: WASI fs mismatch diagnosis (the test's configuration)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06d; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step d1 200 env PIN=1 REP=39 HT=8 python -u tools/wasi_fs_diff.py
step d2 200 env REP=39 HT=0 python -u tools/wasi_fs_diff.py
step d3 200 env REP=3 HT=8 python -u tools/wasi_fs_diff.py
echo all done
