# A/B of the launch plan on whole BASELINE workloads: lane run length L (digits
# enumerated per lane), minimum lanes per bucket and nonces per launch.  Run on the GPU box.
set -u
OUT=gpurun_out/${TAG:-r02ap}; mkdir -p $OUT
M=MINEHIP_LOWER_DIGITS=3,MINEHIP_MIN_LANES=2097152
V="--rounds 3 --var cur: --var L3n34:$M,MINEHIP_LAUNCH_NONCES=17179869184 --var L3n33:$M,MINEHIP_LAUNCH_NONCES=8589934592 --var L3n32:$M,MINEHIP_LAUNCH_NONCES=4294967296"
A=$(printf 'a%.0s' $(seq 100)); X=$(printf 'x%.0s' $(seq 60))
i=0
for args in "--msg cmu440 --lo 0 --count 4294967296" "--msg $A --lo 0 --count 17179869184" \
            "--msg $X --lo 0 --count 17179869184" "--msg cmu440 --lo 549755813888 --count 54975581388"; do
  i=$((i+1))
  timeout -k 10 400 python tools/kbench.py $args $V > $OUT/P$i.json 2> $OUT/P$i.err
  rc=$?; echo "P$i rc=$rc $args" | cut -c1-40; cat $OUT/P$i.json
  [ $rc -eq 0 ] || exit $rc
done
