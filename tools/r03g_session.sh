# round 3: post-RA schedules that alternate half- and full-rate runs (tools/sched_pass.py, R = 1..3)
set -u
O=gpurun_out/r03g; mkdir -p $O
V="--var product:"
for v in prio sched_1_1 sched_1_2 sched_2_1 sched_2_2 sched_3_2 sched_1_3; do V="$V --var $v:MINEHIP_DEV_CODE_OBJECT=build/ab/$v.hsaco"; done
timeout -k 10 300 python tools/kbench.py --lo 1000000000 --count 4294967296 --rounds 7 $V > $O/kbench_d10_sched.json 2> $O/kbench_d10.err || exit $?
timeout -k 10 300 python tools/kbench.py --lo 100000000 --count 900000000 --rounds 7 $V > $O/kbench_d9_sched.json 2> $O/kbench_d9.err || exit $?
echo done
