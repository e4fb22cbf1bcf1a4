set -e
bash tools/gpu_run.sh "tests:lazy_dp or chain_batch or c3_hg38 or golden or round4 or dense or c2_ecoli" r4j
DIRS=". .ab/h0" N=3 bash tools/gpu_run.sh abdir r4j
bash tools/gpu_run.sh s1 r4j
