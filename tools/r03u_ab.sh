# round 3: fast launches as work queues (workgroups claim 256-run chunks from a counter, so the
# XCDs -- whose clocks differ by 2-4% -- finish together) against one chunk per workgroup:
# the same code object both ways (MINEHIP_QUEUE), and the previous build's static code object
set -u
O=gpurun_out/r03u; mkdir -p $O
V="--var static:MINEHIP_QUEUE=0 --var queue:MINEHIP_QUEUE=1 --var old:MINEHIP_QUEUE=0,MINEHIP_DEV_CODE_OBJECT=build/ab/split3_static_old.hsaco"
A=$(printf 'a%.0s' $(seq 100)); X=$(printf 'x%.0s' $(seq 60))
timeout -k 10 400 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 7 --clock $V > $O/d10.json 2> $O/d10.err || exit $?
timeout -k 10 400 python tools/kbench.py --lo 0 --count 4294967296 --rounds 9 $V > $O/cfg1.json 2> $O/cfg1.err || exit $?
timeout -k 10 400 python tools/kbench.py --msg $A --lo 0 --count 17179869184 --rounds 5 $V > $O/cfg3a.json 2> $O/cfg3a.err || exit $?
timeout -k 10 400 python tools/kbench.py --msg $X --lo 0 --count 17179869184 --rounds 5 $V > $O/cfg3b.json 2> $O/cfg3b.err || exit $?
MINEHIP_QUEUE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_parity_queue.log 2>&1 || { tail -20 $O/pytest_parity_queue.log; exit 1; }
tail -2 $O/pytest_parity_queue.log
echo done
