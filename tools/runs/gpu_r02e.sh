set -e
timeout -k 10 300 python bench.py > gpurun_out/r02e_bench_c2.json 2> gpurun_out/r02e_bench_c2.err
for n in 32768 16384 8192; do
  timeout -k 10 120 python bench.py --instances $n --no-cpu-baseline --steps 5 > gpurun_out/r02e_strong_$n.json 2>/dev/null
done
