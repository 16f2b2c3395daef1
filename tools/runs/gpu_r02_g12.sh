set -o pipefail
for pc in 13 153 229 264 350; do echo "== WB_SCAN=$pc"; WB_SCAN=$pc timeout -k 10 120 python -u tools/scan_probe.py 9 4 2>&1 | tail -3 || exit 1; done
