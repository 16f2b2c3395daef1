# r06 g: the whole -m gpu suite at HEAD (trip batching + function guards + one-branch tail,
# WASI subset, stack bound), smoke(), then A/B of the function guards
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06g; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step suite 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step c3k_g1 200 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c3k_g0 200 env WB_TRIP_GUARD=0 python bench.py --workload c3 --elements 4096 --no-cpu-baseline
step c4_g1 200 python bench.py --workload c4 --no-cpu-baseline
step c3_g1 300 python bench.py --workload c3 --no-cpu-baseline
echo all done
