# r03 closing E: the whole -m gpu suite and smoke() at HEAD, the default bench line, C5's
# line with its CPU baseline and C5's rocprofv3 passes
O=gpurun_out/r03z; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step c2 200 python bench.py
step c5 200 python bench.py --workload c5 --instances 262144 --steps 5 --warmup 1
step c4 200 python bench.py --workload c4 --steps 3 --warmup 1
step mt 200 python bench.py --workload mt --steps 2 --warmup 1
export PROF_TIMEOUT=120
step prof_c5 400 bash tools/prof_bench.sh gpurun_out/r03z/pc5 --workload c5 --instances 262144 --steps 3 --warmup 1
