# Workgroups-per-launch A/B (MINEHIP_MAX_BLOCKS), kbench.py per line.
set -e
mkdir -p gpurun_out/r01zo
O=gpurun_out/r01zo/blocks.jsonl
k() { timeout -k 10 200 python tools/kbench.py --rounds 4 "$@" --var b64k: --var b128k:MINEHIP_MAX_BLOCKS=131072 --var b256k:MINEHIP_MAX_BLOCKS=262144 >> $O; }
k --msg cmu440 --lo 0 --count 4294967296
k --msg cmu440 --lo 1000000000 --count 3294967296
k --msg aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa --lo 0 --count 17179869184
