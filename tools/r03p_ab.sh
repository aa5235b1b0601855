# round 3: the add3-split build (product, ADD3_SPLIT=3) against the round-3 build without it
# (build/ab/prio.hsaco), d = 10 bucket with in-kernel clocks and the whole configs[1] search
set -u
O=gpurun_out/r03p; mkdir -p $O
V="--var product: --var nosplit:MINEHIP_DEV_CODE_OBJECT=build/ab/prio.hsaco"
timeout -k 10 400 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 7 --clock $V > $O/kbench_d10.json 2> $O/kbench_d10.err || exit $?
timeout -k 10 400 python tools/kbench.py --lo 0 --count 4294967296 --rounds 9 $V > $O/kbench_cfg1.json 2> $O/kbench_cfg1.err || exit $?
echo done
