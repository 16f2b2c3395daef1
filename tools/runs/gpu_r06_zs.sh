# r06 zs: closing bench lines for the configs without trip mode (C2, C1, C5, tail calls) at
# the final HEAD, so that every r06_end_bench line comes from one build
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zs; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step c2 200 python bench.py
step c1 200 python bench.py --workload c1
step c5 300 python bench.py --workload c5
step tail 200 python bench.py --workload tail
echo all done
