# r05 b: the host-cost test, then what r05 a did not reach: bench lines for C2, C5 and mt
# (repeated and fresh inputs) and the hash kernel's trace + FETCH_SIZE on C3 4K
O=gpurun_out/r05b; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 300 python -u -m pytest tests/test_hostcost.py -m gpu -v --timeout 300 --timeout-method thread
step c2 200 python bench.py --no-cpu-baseline
step c5 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline
step mt 300 python bench.py --workload mt --steps 3 --warmup 4 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step hash_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/hash_trace -o run -- python3 $R/bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
step hash_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/hash_fetch -o run -- python3 $R/bench.py --workload c3 --elements 4096 --steps 2 --warmup 1 --no-cpu-baseline
echo all done
