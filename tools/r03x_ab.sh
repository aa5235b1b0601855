# round 3: with work-queue launches, do the two streams and the 2^28 tail split still pay?
set -u
O=gpurun_out/r03x; mkdir -p $O
V="--var default: --var s1:MINEHIP_STREAMS=1,MINEHIP_FINE_TAIL=0 --var s2t0:MINEHIP_FINE_TAIL=0 --var s2t27:MINEHIP_FINE_TAIL=134217728 --var s2t29:MINEHIP_FINE_TAIL=536870912"
X=$(printf 'x%.0s' $(seq 60))
timeout -k 10 400 python tools/kbench.py --lo 0 --count 4294967296 --rounds 9 $V > $O/cfg1.json 2> $O/cfg1.err || exit $?
timeout -k 10 400 python tools/kbench.py --msg $X --lo 0 --count 17179869184 --rounds 5 $V > $O/cfg3b.json 2> $O/cfg3b.err || exit $?
timeout -k 10 400 python tools/kbench.py --lo 549755813888 --count 68719476736 --rounds 3 $V > $O/cfg4slice.json 2> $O/cfg4slice.err || exit $?
echo done
