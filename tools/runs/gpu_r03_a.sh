# r03 first call: the box's counter list, then the GPU suite at HEAD
set -o pipefail
mkdir -p gpurun_out/r03a
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r03a/counters.txt 2>&1 || echo "list rc=$?"
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03a/tests.log 2>&1 || { tail -30 gpurun_out/r03a/tests.log; exit 3; }
tail -1 gpurun_out/r03a/tests.log
