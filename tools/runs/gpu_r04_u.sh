# r04 u: closing rocprofv3 evidence for C3 at configs[2] size (64K x 1 MiB; warmup 2 so the
# timed launch is past the layout trial), and C3 4K's HBM traffic at 32/64/128-byte granules
# (write amplification by granule)
O=gpurun_out/r04u; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=200
for g in 128 64 32; do
  step g$g 400 env WB_GRANULE=$g PROF_PASSES="trace fetch write" bash tools/prof_bench.sh gpurun_out/r04u/c3k_g$g --workload c3 --elements 4096 --steps 2 --warmup 1
done
step prof_c3 1000 bash tools/prof_bench.sh gpurun_out/r04u/c3 --workload c3 --steps 1 --warmup 2
