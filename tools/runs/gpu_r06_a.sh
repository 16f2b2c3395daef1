# r06 a: WASI prestat + hello.wasm, bounded stack growth / shrink at Reset, LtF wrap fix,
# externref table exhaustion; the default bench line
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06a; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step new 600 python -u -m pytest tests/test_wasi_programs.py tests/test_deepstack.py tests/test_wasi.py tests/test_tripcache.py tests/test_abi.py -m gpu -v --timeout 300 --timeout-method thread
step bench 300 python bench.py
step bench_c3 400 python bench.py --workload c3 --steps 2 --warmup 1
echo all done
