# round 3: the add3 split on every BASELINE layout (wall clock, medians of 7, one process each)
set -u
O=gpurun_out/r03o; mkdir -p $O
V="--var product:"
for v in a3split3 a3split4 a3split5 a3split6 a3split8; do V="$V --var $v:MINEHIP_DEV_CODE_OBJECT=build/ab/$v.hsaco"; done
A=$(printf 'a%.0s' $(seq 100)); X=$(printf 'x%.0s' $(seq 60))
timeout -k 10 400 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 7 --clock $V > $O/d10.json 2> $O/d10.err || exit $?
timeout -k 10 400 python tools/kbench.py --lo 100000000 --count 900000000 --rounds 7 $V > $O/d9.json 2> $O/d9.err || exit $?
timeout -k 10 400 python tools/kbench.py --lo 0 --count 4294967296 --rounds 7 $V > $O/cfg1.json 2> $O/cfg1.err || exit $?
timeout -k 10 400 python tools/kbench.py --msg $A --lo 0 --count 17179869184 --rounds 5 $V > $O/cfg3a.json 2> $O/cfg3a.err || exit $?
timeout -k 10 400 python tools/kbench.py --msg $X --lo 0 --count 17179869184 --rounds 5 $V > $O/cfg3b.json 2> $O/cfg3b.err || exit $?
echo done
