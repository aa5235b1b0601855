# round 3: instruction-fetch probe -- the product loop with every k-th s_setprio doubled
# (same issue behaviour, +4 bytes per copy), d = 10 bucket of configs[1], A/B in one process
set -u
O=gpurun_out/r03j; mkdir -p $O
V="--var product:"
for v in prio dup4 dup2 dup1; do V="$V --var $v:MINEHIP_DEV_CODE_OBJECT=build/ab/$v.hsaco"; done
timeout -k 10 300 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 7 $V > $O/kbench_d10_dup.json 2> $O/kbench_d10_dup.err || exit $?
echo done
