# round 3: the add3 split (every k-th v_add3 as two full-rate adds: lower mix bound, more
# instructions) against the product, with each variant's in-kernel clock (kbench --clock)
set -u
O=gpurun_out/r03n; mkdir -p $O
V="--var product:"
for v in a3split2 a3split3 a3split4; do V="$V --var $v:MINEHIP_DEV_CODE_OBJECT=build/ab/$v.hsaco"; done
timeout -k 10 400 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 5 --clock $V > $O/kbench_d10_a3split_clock.json 2> $O/kbench.err || exit $?
echo done
