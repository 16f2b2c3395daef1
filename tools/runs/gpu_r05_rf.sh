# r05 rf: Reset folded into the next interpreter launch (fused_reset): whole -m gpu suite,
# then C2 / C5 with it on and off
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05rf; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-160)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step c2_on 300 python bench.py
step c2_off 300 env WB_FUSED_RESET=0 python bench.py
step c2_on2 300 python bench.py
step c5_on 300 python bench.py --workload c5 --steps 5 --warmup 2
step c5_off 300 env WB_FUSED_RESET=0 python bench.py --workload c5 --steps 5 --warmup 2
echo all done
