set -u
bash tools/gpu_session.sh r03b info tests smoke bench prof || exit $?
O=gpurun_out/r03b
timeout -k 10 300 python tools/kbench.py --lo 0 --count 4294967296 --rounds 5 --var base:MINEHIP_DEV_CODE_OBJECT=build/ab/r03_base.hsaco --var new: --var new_s2:MINEHIP_STREAMS=2 > $O/kbench_cfg1.json 2> $O/kbench_cfg1.err || exit $?
timeout -k 10 300 python tools/kbench.py --lo 1000000 --count 999000000 --rounds 5 --var base:MINEHIP_DEV_CODE_OBJECT=build/ab/r03_base.hsaco --var new: > $O/kbench_d79.json 2> $O/kbench_d79.err || exit $?
timeout -k 10 120 build/valu_ops > $O/valu_ops.json 2>&1 || exit $?
echo done
