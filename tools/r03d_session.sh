# round 3: two-stream execution with the tail split, A/B on every BASELINE workload (wall clock)
set -u
O=gpurun_out/r03d; mkdir -p $O
V="--var s1: --var s2:MINEHIP_STREAMS=2 --var s2t27:MINEHIP_STREAMS=2,MINEHIP_FINE_TAIL=134217728 --var s2t28:MINEHIP_STREAMS=2,MINEHIP_FINE_TAIL=268435456 --var s2t29:MINEHIP_STREAMS=2,MINEHIP_FINE_TAIL=536870912"
for c in "cfg1 cmu440 0 4294967296" "shard8 cmu440 549755813888 6871947673" "cfg3a aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa 0 17179869184" "cfg3b xxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx 0 17179869184"; do
  set -- $c
  timeout -k 10 300 python tools/kbench.py --msg $2 --lo $3 --count $4 --rounds 5 $V > $O/kbench_$1.json 2> $O/kbench_$1.err || exit $?
done
MINEHIP_STREAMS=2 MINEHIP_FINE_TAIL=268435456 timeout -k 10 300 python -u tools/strong_shards.py --ns 1,8 --out $O/strong_s2t28.json > $O/strong_s2t28.log 2>&1 || exit $?
echo done
