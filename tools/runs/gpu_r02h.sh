#!/bin/bash
# r02h: C3 quicksort at the three memory interleave granules (bench + HBM counters), and
# a C2 no-regression bench line. Every GPU step under its own time limit.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/bench.py --no-cpu-baseline --steps 5 > $O/c2.json 2> $O/c2.err
for g in 4 16 128; do
  export WB_GRANULE=$g
  B="$R/bench.py --no-cpu-baseline --workload c3 --elements 16384 --steps 2 --warmup 1"
  timeout -k 10 300 python3 $B > $O/c3_g$g.json 2> $O/c3_g$g.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g$g/trace -o run -- python3 $B > $O/g$g.trace.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/g$g/fetch -o run -- python3 $B > $O/g$g.fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/g$g/write -o run -- python3 $B > $O/g$g.write.log 2>&1
done
echo done
