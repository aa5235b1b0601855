#!/bin/bash
# bench.py's own timed region, A/B: the driver's command (no PMC / CPU baseline / clock / n1 passes)
# run alternately with each variant's environment, ROUNDS times, on one box.
#   bash tools/bench_ab.sh <tag> <rounds> name=K=V,K=V name2= ...
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG; mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    name=${v%%=*}; envs=${v#*=}
    (IFS=,; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
     timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-clock --no-n1 \
         > "$OUT/bench_${name}_$i.json" 2> "$OUT/bench_${name}_$i.err")
    rc=$?; echo "$name round $i rc=$rc $(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" "$OUT/bench_${name}_$i.json" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
