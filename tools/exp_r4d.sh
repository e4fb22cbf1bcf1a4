set -e
DIRS=". .ab/r03" N=2 bash tools/gpu_run.sh "tests:sort or round4 or views or multi_chain,abdir,s1" r4d
AB="-|view_reads=0" N=2 ABSTEPS=10 BARGS="--preset ecoli --reads 1000" bash tools/gpu_run.sh ab r4d_c2
AB="-|mw_min=4096|mw_min=1024" N=1 ABSTEPS=2 BARGS="--reads 2000 --read-len 100000 --warmup 1" bash tools/gpu_run.sh ab r4d_c5
