# r05 x: the whole -m gpu suite and smoke() at HEAD; closing C5 / C2 lines after the parked
# word; the grow workload's same-build profile
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05x; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step c5 300 python bench.py --workload c5 --steps 5 --warmup 2
step c2 300 python bench.py
export PROF_TIMEOUT=240
step prof_c3grow 900 bash $R/tools/prof_bench.sh gpurun_out/r05x/c3grow --workload c3grow --steps 1 --warmup 3
echo all done
