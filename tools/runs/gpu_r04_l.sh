# r04 l: host cost of a bench step (launch + sync overhead) on a trivial module, by batch size
O=gpurun_out/r04l; mkdir -p $O
for n in 64 16384 65536 131072 262144; do
  timeout -k 10 120 python3 tools/host_overhead.py $n > $O/ho$n.log 2>&1 || { cat $O/ho$n.log; exit 1; }
  WB_PERSIST=0 timeout -k 10 120 python3 tools/host_overhead.py $n > $O/ho${n}_np.log 2>&1 || { cat $O/ho${n}_np.log; exit 1; }
done
cd $O && tail -n 3 ho*.log
