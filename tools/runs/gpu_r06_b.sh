# r06 b: QuickJS on the GPU (512 lanes), the WASI fs subset, hello.wasm; C3 at its default
# warm-up (the layout trial outside the timed steps) after the LtF wrap check
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06b; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-300)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step wasi 600 python -u -m pytest tests/test_wasi_fs.py tests/test_quickjs.py tests/test_wasi_programs.py -m gpu -v --timeout 400 --timeout-method thread
step bench_c3 400 python bench.py --workload c3
echo all done
