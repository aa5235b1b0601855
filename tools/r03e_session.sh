set -u
bash tools/gpu_session.sh r03e info tests smoke bench prof latency || exit $?
O=gpurun_out/r03e
timeout -k 10 300 python tools/kbench.py --lo 0 --count 4294967296 --rounds 7 --var new: --var old:MINEHIP_STREAMS=1,MINEHIP_FINE_TAIL=0 > $O/kbench_cfg1_default.json 2> $O/kbench_cfg1_default.err || exit $?
echo done
