#!/bin/bash
# usage: tools/prof_bench.sh <outdir> [bench args...]
# rocprofv3 evidence for bench.py, each collection in its own run (gpurun forbids mixing
# --pmc with tracing): kernel trace + stats of the bench command itself, then FETCH_SIZE,
# WRITE_SIZE (separate passes: TCC slots) and SQ issue counters of the same command.
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/trace -o run -- python3 $B > $R/$OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$OUT/fetch -o run -- python3 $B > $R/$OUT/fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$OUT/write -o run -- python3 $B > $R/$OUT/write.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH --output-format csv -d $R/$OUT/sq1 -o run -- python3 $B > $R/$OUT/sq1.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $R/$OUT/sq2 -o run -- python3 $B > $R/$OUT/sq2.log 2>&1 || exit 5
echo done
