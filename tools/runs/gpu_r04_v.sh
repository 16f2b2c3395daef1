# r04 v: closing bench lines at HEAD with their CPU baselines (rooflines from the r04t/r04u
# profiles of this same build, profiles/prof_<workload>.json)
O=${OUT:-gpurun_out/r04v}; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err; local rc=$?
  echo "$n rc=$rc $(tail -c 300 $O/$n.json)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; tail -5 $O/$n.err; exit $rc; fi
}
step c2 300 python bench.py
step c1 300 python bench.py --workload c1 --steps 3 --warmup 1
step c4 300 python bench.py --workload c4 --steps 10 --warmup 2
step c5 300 python bench.py --workload c5 --instances 262144 --steps 10 --warmup 2
step mt 300 python bench.py --workload mt --steps 5 --warmup 2
step tail 300 python bench.py --workload tail --steps 5 --warmup 2
step c3 600 python bench.py --workload c3 --steps 2 --warmup 2
