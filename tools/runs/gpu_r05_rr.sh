# r05 rr: RET reads its known sites' POST_CALL restores along with the record (Lrp stubs):
# the whole -m gpu suite, then fib latency and C1 with the stubs on / off
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05rr; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step suite 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step fib_on 300 python tools/fib_probe.py
step fib_off 300 env WB_RET_RESTORE=0 python tools/fib_probe.py
step c1_on 300 python bench.py --workload c1
step c1_off 300 env WB_RET_RESTORE=0 python bench.py --workload c1
step c1_on2 300 python bench.py --workload c1
echo all done
