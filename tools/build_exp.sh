# Timing-experiment build: libmm2g_<name>.so with extra -D flags on the kernels (select with MM2G_LIB).
# bash tools/build_exp.sh <name> "-DFOO -DBAR"
set -e
cd "$(dirname "$0")/../minimap2_rs_amd/csrc"
B=../build
mkdir -p $B/exp_$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w $2 -c mm2g_kernels.hip -o $B/exp_$1/k.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libmm2g_$1.so $B/exp_$1/k.o $B/mm2g_host.o $B/mm2g_index.o $B/mm2g_ixbuild.o $B/mm2g_reads.o -pthread
