set -o pipefail
mkdir -p gpurun_out/g5
run() { echo "== $*"; timeout -k 10 60 "$@" > gpurun_out/g5/p.log 2>&1 || { tail -5 gpurun_out/g5/p.log; exit 1; }; grep -E "bad lanes|lane [0-3] " gpurun_out/g5/p.log; }
run python -u tools/simt_probe.py 64 uni
WB_SIMT=0 run python -u tools/simt_probe.py 64
WB_SIMT_X=0 run python -u tools/simt_probe.py 64
WB_SIMT_X=1 run python -u tools/simt_probe.py 64
WB_SIMT_X=2 run python -u tools/simt_probe.py 64
WB_SIMT_X=4 run python -u tools/simt_probe.py 64
run python -u tools/simt_probe.py 2
run python -u tools/simt_probe.py 64
