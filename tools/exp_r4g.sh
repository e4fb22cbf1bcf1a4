set -e
bash tools/gpu_run.sh "tests:filtered_sort or many_shapes or round4 or c3_hg38 or c2_ecoli or golden or wide_gaps or lazy_dp" r4g
bash tools/gpu_run.sh s1 r4g
AB="-|sort_p1count=0" N=3 bash tools/gpu_run.sh ab r4g_ab
