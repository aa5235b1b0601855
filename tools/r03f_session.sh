set -u
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread -k "not config5" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/gpu_session.sh r03f smoke bench prof latency || exit $?
python tools/trace_frac.py $O/prof_bench.json $O/prof/run_kernel_trace.csv > $O/trace_frac.json
timeout -k 10 300 python tools/kbench.py --lo 0 --count 4294967296 --rounds 7 --var new: --var old:MINEHIP_STREAMS=1,MINEHIP_FINE_TAIL=0 > $O/kbench_cfg1_default.json 2> $O/kbench_cfg1_default.err || exit $?
echo done
