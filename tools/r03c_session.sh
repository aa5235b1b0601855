# round 3: code-object alignment / register / compare-class A/B on the d = 10 bucket, and the
# two-stream execution on every BASELINE workload (wall clock)
set -u
O=gpurun_out/r03c; mkdir -p $O
V=""
for v in pad0 pad1 pad2 pad4 pad8 pad12 cmpH r03_base; do V="$V --var $v:MINEHIP_DEV_CODE_OBJECT=build/ab/$v.hsaco"; done
timeout -k 10 300 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 7 $V > $O/kbench_d10_variants.json 2> $O/kbench_d10.err || exit $?
for c in "cfg1 cmu440 0 4294967296" "cfg3a aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa 0 17179869184" "cfg3b xxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx 0 17179869184" "cfg4slice cmu440 549755813888 68719476736"; do
  set -- $c
  timeout -k 10 300 python tools/kbench.py --msg $2 --lo $3 --count $4 --rounds 5 --var s1: --var s2:MINEHIP_STREAMS=2 > $O/kbench_streams_$1.json 2> $O/kbench_streams_$1.err || exit $?
done
echo done
