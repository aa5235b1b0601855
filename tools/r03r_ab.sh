# round 3: which add3s to split -- every third in program order (the build) against the ones
# whose results are read latest (a3far<pct>: the pct% with the most slack)
set -u
O=gpurun_out/r03r; mkdir -p $O
V="--var product:"
for v in a3far25 a3far33 a3far40; do V="$V --var $v:MINEHIP_DEV_CODE_OBJECT=build/ab/$v.hsaco"; done
X=$(printf 'x%.0s' $(seq 60))
timeout -k 10 400 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 7 --clock $V > $O/d10.json 2> $O/d10.err || exit $?
timeout -k 10 400 python tools/kbench.py --lo 0 --count 4294967296 --rounds 7 $V > $O/cfg1.json 2> $O/cfg1.err || exit $?
timeout -k 10 400 python tools/kbench.py --msg $X --lo 0 --count 17179869184 --rounds 5 $V > $O/cfg3b.json 2> $O/cfg3b.err || exit $?
echo done
