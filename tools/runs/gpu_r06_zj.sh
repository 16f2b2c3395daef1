# r06 zj: closing bench lines at HEAD (after the trip-chain changes), one per config, each with its CPU baseline (the oracle
# on the box's host threads, bit-exact against the GPU on its sample) and rooflines from the
# same build's profiles (profiles/prof_<config>.json)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zj; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step c2 200 python bench.py
step c1 200 python bench.py --workload c1
step c4 200 python bench.py --workload c4
step c5 300 python bench.py --workload c5
step mt 300 python bench.py --workload mt
step tail 200 python bench.py --workload tail
step c3 300 python bench.py --workload c3
step c3x 300 python bench.py --workload c3x
step c3grow 300 python bench.py --workload c3grow
echo all done
