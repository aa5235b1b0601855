#!/bin/bash
# Launch-plan A/B experiments behind DESIGN.md §3 (profiles/r01zg..r01zo).  Every line is one
# tools/kbench.py process that interleaves its variants (env settings of the planner knobs) round
# by round, so each A/B shares one box and one clock.  kbench's GH/s is nonces / summed kernel
# time (HIP events), i.e. launch gaps excluded.
#   bash tools/plan_ab.sh <tag> [size|lanes|defaults|blocks]
set -e
TAG=${1:-r01zx}; WHAT=${2:-defaults}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
A100=$(python -c "print('a' * 100)")
X60=$(python -c "print('x' * 60)")
k() { timeout -k 10 200 python tools/kbench.py "$@" >> "$OUT/$WHAT.jsonl"; }
case $WHAT in
  size)      # one d = 10 launch of 2^29..2^33 nonces at L = 3 (r01zg)
    for c in 29 30 31 32 33; do
      k --lo 1000000000 --count $((1 << c)) --rounds 3 --var "c$c:MINEHIP_LOWER_DIGITS=3,MINEHIP_LAUNCH_NONCES=$((1 << 33))"
    done ;;
  lanes)     # lower-digit count per bucket (r01zi..r01zk)
    k --msg cmu440 --lo 1000000000 --count 3294967296 --rounds 3 \
      --var L3:MINEHIP_LOWER_DIGITS=3 --var L2:MINEHIP_LOWER_DIGITS=2 --var L1:MINEHIP_LOWER_DIGITS=1
    k --msg cmu440 --lo 20000000000 --count 17179869184 --rounds 3 \
      --var L3:MINEHIP_LOWER_DIGITS=3 --var L2:MINEHIP_LOWER_DIGITS=2 \
      --var L3big:MINEHIP_LOWER_DIGITS=3,MINEHIP_LAUNCH_NONCES=17179869184 ;;
  defaults)  # old plan (L <= 3, 2^18 lanes, 65,536 workgroups) against the current one (r01zl)
    OLD=old:MINEHIP_LOWER_DIGITS=3,MINEHIP_MIN_LANES=262144,MINEHIP_MAX_BLOCKS=65536
    for args in "--msg cmu440 --lo 0 --count 4294967296" "--msg $A100 --lo 0 --count 17179869184" \
                "--msg $X60 --lo 0 --count 17179869184" "--msg cmu440 --lo 0 --count 100000000"; do
      k $args --rounds 4 --var "$OLD" --var new:
    done ;;
  blocks)    # workgroups per launch (r01zo)
    for args in "--msg cmu440 --lo 0 --count 4294967296" "--msg cmu440 --lo 1000000000 --count 3294967296"; do
      k $args --rounds 4 --var b64k:MINEHIP_MAX_BLOCKS=65536 --var b128k:MINEHIP_MAX_BLOCKS=131072 \
        --var b256k:MINEHIP_MAX_BLOCKS=262144
    done ;;
  *) echo "unknown experiment $WHAT"; exit 2 ;;
esac
cat "$OUT/$WHAT.jsonl"
