set -u
OUT=gpurun_out/r02ak; mkdir -p $OUT
V="--rounds 3 --var prio:MINEHIP_DEV_CODE_OBJECT=build/isa/prio.hsaco --var grp_ilp:MINEHIP_DEV_CODE_OBJECT=build/isa/grp_ilp.hsaco"
i=0
for args in "--msg cmu440 --lo 1000000000 --count 2147483648" \
            "--msg aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa --lo 10000000000 --count 4294967296" \
            "--msg xxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxxx --lo 10000000000 --count 2147483648" \
            "--msg cmu440-cmu440-cmu440-cmu440-cmu440-cmu440-cmu440-cmu --lo 1000000000 --count 1073741824" \
            "--msg cmu440 --lo 100000000 --count 805306368"; do
  i=$((i+1))
  timeout -k 10 300 python tools/kbench.py $args $V > $OUT/ab$i.json 2> $OUT/ab$i.err
  rc=$?; echo "ab$i rc=$rc $args" | cut -c1-80; cat $OUT/ab$i.json
  [ $rc -eq 0 ] || exit $rc
done
