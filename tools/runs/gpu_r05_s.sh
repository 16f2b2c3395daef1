# r05 s: closing rocprofv3 evidence for C3 at configs[2] size (64K x 1 MiB; warmup 3: the
# timed launch is past the layout trial) after the trip shortcuts
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05s; mkdir -p $O
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc $(tail -1 $O/$n.log | cut -c1-150)"
  if [ $rc -ne 0 ]; then echo "stopping after $n"; exit $rc; fi
}
export PROF_TIMEOUT=240
step prof_c3 1150 bash $R/tools/prof_bench.sh gpurun_out/r05s/c3 --workload c3 --steps 1 --warmup 3
