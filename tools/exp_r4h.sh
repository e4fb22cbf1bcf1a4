set -e
DIRS=". .ab/r03" N=2 ABSTEPS=2 BARGS="--reads 2000 --read-len 100000 --warmup 1" bash tools/gpu_run.sh abdir r4h_c5
O=gpurun_out/r4h_c5
for D in . .ab/r03; do
  nm=$(echo "$D" | tr -c 'a-zA-Z0-9\n' '_')
  (cd "$D" && timeout -k 10 300 python -u bench.py --reads 2000 --read-len 100000 --steps 1 --warmup 0 --streams 1 --shares 1 --no-cpu --no-parity --resident-steps 0 --knob sort_prof=1) > $O/c5s1_$nm.json 2> $O/c5s1_$nm.err
  grep sort_prof $O/c5s1_$nm.err | tail -3 || true
done
