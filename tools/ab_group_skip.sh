# A/B: group-level recompute only when word J-1 changes (product build) against the previous
# code object (build/old_prio.hsaco), whole searches, one process each.
set -u
OUT=gpurun_out/${TAG:-r02as}; mkdir -p $OUT
V="--rounds 3 --var new: --var old:MINEHIP_DEV_CODE_OBJECT=build/old_prio.hsaco"
A=$(printf 'a%.0s' $(seq 100)); X=$(printf 'x%.0s' $(seq 60)); P=$(python3 -c 'print(("cmu440-"*10)[:55])')
i=0
for args in "--msg cmu440 --lo 549755813888 --count 54975581388" "--msg cmu440 --lo 0 --count 4294967296" \
            "--msg $A --lo 0 --count 17179869184" "--msg $X --lo 0 --count 17179869184" \
            "--msg $P --lo 0 --count 4294967296"; do
  i=$((i+1))
  timeout -k 10 400 python tools/kbench.py $args $V > $OUT/G$i.json 2> $OUT/G$i.err
  rc=$?; echo "G$i rc=$rc $args" | cut -c1-50; cat $OUT/G$i.json
  [ $rc -eq 0 ] || exit $rc
done
