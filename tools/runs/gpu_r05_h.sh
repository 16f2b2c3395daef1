# r05 h: reserved layout grown at Reset to the pages the lanes reached; memgrow tests and the
# C3 / growing-C3 benches
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05h; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}

step tests 600 python -u -m pytest tests/test_memgrow.py tests/test_layout.py tests/test_multidevice.py tests/test_hostcall.py -m gpu -v --timeout 300 --timeout-method thread
step c3k 300 python bench.py --workload c3 --elements 4096 --steps 3 --warmup 3 --no-cpu-baseline
step c3gk 300 python bench.py --workload c3grow --elements 4096 --steps 3 --warmup 3 --no-cpu-baseline
step knobs 300 python3 $R/tools/c3_writes.py --only base,trip0,scan0,chain0,split0,hyb0
cd /tmp && export TMPDIR=/tmp
step write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/tools/c3_writes.py --only base,trip0,scan0,chain0,split0,hyb0
cd $R
step c3 400 python bench.py --workload c3 --steps 2 --warmup 3 --no-cpu-baseline
step c3g 400 python bench.py --workload c3grow --steps 2 --warmup 3 --no-cpu-baseline
echo all done
