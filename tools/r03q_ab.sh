# round 3: which add3s to split -- the build's every-third (001) against other phases and ratios
set -u
O=gpurun_out/r03q; mkdir -p $O
V="--var product:"
for v in a3pat010 a3pat100 a3pat01 a3pat00101 a3pat0001001; do V="$V --var $v:MINEHIP_DEV_CODE_OBJECT=build/ab/$v.hsaco"; done
X=$(printf 'x%.0s' $(seq 60))
timeout -k 10 400 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 7 $V > $O/d10.json 2> $O/d10.err || exit $?
timeout -k 10 400 python tools/kbench.py --lo 0 --count 4294967296 --rounds 7 $V > $O/cfg1.json 2> $O/cfg1.err || exit $?
timeout -k 10 400 python tools/kbench.py --msg $X --lo 0 --count 17179869184 --rounds 5 $V > $O/cfg3b.json 2> $O/cfg3b.err || exit $?
echo done
