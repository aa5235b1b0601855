#!/bin/bash
# Samples the GPU's power and clocks (amd-smi) while the fast kernel runs, to tell a power-capped
# clock from an issue-bound loop.  Usage: bash tools/power_probe.sh <tag> [kbench args]
set -u
TAG=${1:-r02u}; shift || true
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
(amd-smi static --limit 2>&1; amd-smi static --clock 2>&1) > "$OUT/limits.txt"
timeout -k 10 120 python tools/kbench.py --lo 100000000000 --count 68719476736 --rounds 12 "$@" > "$OUT/kbench.json" 2> "$OUT/kbench.err" &
pid=$!
sleep 6
for i in 1 2 3 4 5 6; do
  amd-smi metric --power --clock --temperature 2>&1 >> "$OUT/metric.txt"
  echo "----" >> "$OUT/metric.txt"
  sleep 2
done
wait $pid
echo "kbench rc=$?"
cat "$OUT/kbench.json"
