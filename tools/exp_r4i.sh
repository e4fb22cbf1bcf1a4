set -e
bash tools/gpu_run.sh "tests:filtered_sort or many_shapes or c5_hg38 or c3_hg38 or golden or round4" r4i
DIRS=". .ab/h0" N=2 bash tools/gpu_run.sh abdir r4i_c3
DIRS=". .ab/h0" N=2 ABSTEPS=2 BARGS="--reads 2000 --read-len 100000 --warmup 1" bash tools/gpu_run.sh abdir r4i_c5
O=gpurun_out/r4i_c5
timeout -k 10 300 python -u bench.py --reads 2000 --read-len 100000 --steps 1 --warmup 0 --streams 1 --shares 1 --no-cpu --no-parity --resident-steps 0 --knob sort_prof=1 > $O/c5s1.json 2> $O/c5s1.err
grep "sort_prof\] reads" $O/c5s1.err || true
timeout -k 10 300 python -u bench.py --no-cpu --no-parity --resident-steps 0 --steps 1 --warmup 0 --streams 1 --shares 1 --knob sort_prof=1 > $O/c3s1.json 2> $O/c3s1.err
grep "sort_prof\] reads" $O/c3s1.err || true
