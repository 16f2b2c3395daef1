# r06 zx: closing bench lines for the trip-mode configs at the final HEAD (trips left only
# when no lane is in them), then the whole -m gpu suite and smoke()
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zx; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step c4 200 python bench.py --workload c4
step mt 300 python bench.py --workload mt
step c3 300 python bench.py --workload c3
step c3x 300 python bench.py --workload c3x
step c3grow 300 python bench.py --workload c3grow
step suite 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
echo all done
