# r06 p: C5 / mt fresh inputs with the last launch's wave order reused on new arguments
# (WB_ORDER_ANY=1) against the default; C1 after the pc-0 re-aim trim
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06p; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step c5_def 300 python bench.py --workload c5 --no-cpu-baseline
step c5_any 300 env WB_ORDER_ANY=1 python bench.py --workload c5 --no-cpu-baseline
step mt_any 300 env WB_ORDER_ANY=1 python bench.py --workload mt --no-cpu-baseline
step c1 300 python bench.py --workload c1 --no-cpu-baseline
echo all done
