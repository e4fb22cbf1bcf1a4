set -e
bash tools/gpu_run.sh "tests:round4 or filtered_sort or many_shapes or views or c3_hg38 or sketch_parity" r4f
DIRS=". .ab/r03" N=3 bash tools/gpu_run.sh abdir r4f
AB="-|sort_lb=1" N=2 bash tools/gpu_run.sh ab r4f_ab
BARGS="--knob sort_lb=1" bash tools/gpu_run.sh s1 r4f_lb1
