# r06 zk: the whole -m gpu suite and smoke() at the closing HEAD
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zk; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step suite 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
echo all done
