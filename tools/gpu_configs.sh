# C2 (E. coli, 1000 x 10 kb) and C5 (hg38, 2000 x 100 kb) bench lines with the oracle parity check.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --preset ecoli --reads 1000 --steps 10 --warmup 2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
timeout -k 10 500 python bench.py --reads 2000 --read-len 100000 --steps 3 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
