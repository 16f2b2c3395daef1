#!/bin/bash
# usage: tools/prof_bench.sh <outdir> [bench args...]
# rocprofv3 evidence for one bench.py configuration, each collection in its own run (gpurun
# forbids mixing --pmc with tracing; one pass per counter group, MI355X_MICROARCH.md):
#   trace  kernel trace + stats of the bench command itself (kernel durations)
#   fetch  FETCH_SIZE        write  WRITE_SIZE          (HBM bytes, separate TCC passes)
#   sq1    issue counts: waves, wave cycles, VALU / SALU / SMEM / LDS / branch instructions
#   sq2    where wave cycles go: active / waiting, VMEM instructions, GRBM_GUI_ACTIVE
#   util   SQ_THREAD_CYCLES_VALU (active lanes per VALU instruction = exec-mask efficiency),
#          L2 hits / misses
#   lat    VmemLatency (mean cycles a vector-memory instruction is in flight)
# PROF_PASSES="trace fetch ..." runs a subset. Summarise with tools/prof_summary.py.
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline $*"
T=${PROF_TIMEOUT:-300}
PASSES=${PROF_PASSES:-"trace fetch write sq1 sq2 util lat"}
k=0
for p in $PASSES; do
  k=$((k + 1))
  case $p in
    trace) A="--kernel-trace --stats" ;;
    fetch) A="--pmc FETCH_SIZE" ;;
    write) A="--pmc WRITE_SIZE" ;;
    sq1) A="--pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH" ;;
    sq2) A="--pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" ;;
    util) A="--pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum" ;;
    lat) A="--pmc VmemLatency" ;;
    *) echo "unknown pass $p"; exit 9 ;;
  esac
  echo "[prof] pass $p" >&2
  timeout -k 10 $T rocprofv3 $A --output-format csv -d $R/$OUT/$p -o run -- python3 $B > $R/$OUT/$p.log 2>&1 || { echo "pass $p failed"; tail -5 $R/$OUT/$p.log; exit $k; }
done
echo done
