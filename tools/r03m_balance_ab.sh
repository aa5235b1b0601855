# round 3: 8 launched ranks on the box's one GPU, configs[3] layout at 2^36: equal shards
# (BENCH_BALANCE=0) against rate-balanced shards, alternating, same box
set -u
O=gpurun_out/r03m; mkdir -p $O
for i in 1 2; do
  for b in 0 1; do
    BENCH_BALANCE=$b BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port $((29600 + 2 * i + b)) bench.py --gpus 8 --steps 8 --warmup 2 \
        --bits 36 --no-clock > $O/dist8_b${b}_$i.json 2> $O/dist8_b${b}_$i.err || exit $?
  done
done
echo done
