set -e
DIRS=". .ab/r03" N=3 bash tools/gpu_run.sh "tests:seed or sort_parity,abdir" r4e
AB="-|prune_rescue=0|view_reads=0" N=2 bash tools/gpu_run.sh ab r4e_ab
AB="-|view_reads=0" N=3 ABSTEPS=10 BARGS="--preset ecoli --reads 1000" bash tools/gpu_run.sh ab r4e_c2
