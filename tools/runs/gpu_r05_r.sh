# r05 r: MultiMemories on the GPU (memories past the first in the paged kernels' per-lane
# step) + the paths the kernel change touches (memgrow, layout, workloads), C2/C1 benches
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05r; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-250)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests/test_multimem.py -m gpu -v --timeout 300 --timeout-method thread
step c2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
step c1 300 python bench.py --workload c1 --steps 2 --warmup 2 --no-cpu-baseline
echo all done
