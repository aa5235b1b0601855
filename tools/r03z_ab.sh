# round 3: the work-queue build's per-layout register caps (min_waves) against no cap
# (MH_MIN_WAVES=1: more VGPRs -> fewer waves, but no SGPR squeeze -> no s_mov in the loop)
set -u
O=gpurun_out/r03z; mkdir -p $O
V="--var product: --var w1:MINEHIP_DEV_CODE_OBJECT=build/ab/queue_w1.hsaco"
A=$(printf 'a%.0s' $(seq 100)); X=$(printf 'x%.0s' $(seq 60))
timeout -k 10 400 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 9 --clock $V > $O/d10.json 2> $O/d10.err || exit $?
timeout -k 10 400 python tools/kbench.py --lo 0 --count 4294967296 --rounds 9 $V > $O/cfg1.json 2> $O/cfg1.err || exit $?
timeout -k 10 400 python tools/kbench.py --msg $A --lo 0 --count 17179869184 --rounds 5 $V > $O/cfg3a.json 2> $O/cfg3a.err || exit $?
timeout -k 10 400 python tools/kbench.py --msg $X --lo 0 --count 17179869184 --rounds 5 $V > $O/cfg3b.json 2> $O/cfg3b.err || exit $?
echo done
