# One vs two launch streams (MINEHIP_STREAMS): bench.py wall clock, interleaved runs.
set -e
mkdir -p gpurun_out/r01zs
for i in 1 2 3; do
  for s in 1 2; do
    MINEHIP_STREAMS=$s timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/r01zs/s${s}_$i.json
  done
done
