# r05 fin (reuses the r05 z recipe): closing run at HEAD -- metered table widening, the whole -m gpu suite, smoke(),
# the default bench line
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05fin; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tables 300 python -u -m pytest tests/test_tables.py -m gpu -v --timeout 200 --timeout-method thread
step suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py
echo all done
