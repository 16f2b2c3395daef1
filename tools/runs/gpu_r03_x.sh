# r03 closing D: the whole -m gpu suite, smoke() and the default bench line at HEAD (what
# the driver runs), C1's line with its CPU baseline, and C1's rocprofv3 passes at HEAD
O=gpurun_out/r03x; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step c2 200 python bench.py
step c1 200 python bench.py --workload c1 --steps 3 --warmup 1
export PROF_TIMEOUT=120
step prof_c1 400 bash tools/prof_bench.sh gpurun_out/r03x/pc1 --workload c1 --steps 1 --warmup 0
