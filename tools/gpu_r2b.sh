# BASELINE-config GPU tests, then bench variants (streams x pack threads), no CPU leg.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_configs.py > gpurun_out/t2.log 2>&1 || echo "configs failed rc=$?" >> gpurun_out/t2.log
for s in 2 3; do for p in 4 8; do
  timeout -k 10 300 python -u bench.py --no-parity --resident-steps 0 --streams $s --pack-threads $p > gpurun_out/b_s${s}_p${p}.json 2> gpurun_out/b_s${s}_p${p}.err
done; done
