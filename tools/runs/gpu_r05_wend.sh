# r05 w: the closing bench line of every config at HEAD (after table widening, 64-bit externrefs, the fused reset)
# oracle on the box's host cores, bit-exact against the GPU on its sample) and rooflines
# from the same build's profiles (r05q); C5 and mt also on fresh inputs per step
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05wend; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
step c2 300 python bench.py
step c1 300 python bench.py --workload c1 --steps 2 --warmup 2
step c4 300 python bench.py --workload c4 --steps 10 --warmup 5
step c5 300 python bench.py --workload c5 --steps 5 --warmup 2
step mt 300 python bench.py --workload mt --steps 3 --warmup 3
step tail 300 python bench.py --workload tail --steps 3 --warmup 2
step c3 500 python bench.py --workload c3 --steps 2 --warmup 3
step c3grow 500 python bench.py --workload c3grow --steps 2 --warmup 3
echo all done
