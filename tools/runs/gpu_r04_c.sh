# r04 c: per-wave timelines (stats build) of the divergent configs
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 500 python -u tools/wave_timeline.py c1 c4 c5 c3 --out $O/timeline.json > $O/timeline.log 2>&1; rc=$?
tail -5 $O/timeline.log; exit $rc
