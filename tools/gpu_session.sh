#!/bin/bash
# One GPU-box session: parity tests, bench, rocprof kernel-trace summary.
# Each GPU step runs under its own timeout; after a crash / abort / timeout
# (exit 124, 134, 137, 139 or >128) nothing else touches the GPU.
# Usage (from the repo root on the box): bash tools/gpu_session.sh [TAG] [STEPS...]
#   STEPS default: info tests bench prof
set -u
TAG=${1:-r01}; shift || true
STEPS=${*:-info tests bench prof}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

fatal() { # exit code -> 0 if it is safe to continue on the GPU
  local rc=$1
  if [ "$rc" -eq 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 137 ] || [ "$rc" -eq 139 ] || [ "$rc" -gt 128 ]; then
    echo "GPU step ended with $rc: stopping the session" | tee -a "$OUT/session.log"; exit "$rc"
  fi
}

for s in $STEPS; do
  echo "== $s $(date +%T)" | tee -a "$OUT/session.log"
  case $s in
    info)
      (rocminfo 2>&1 | grep -E 'Marketing Name|Name: +gfx|Compute Unit|Max Clock|SIMDs per CU' | head -20
       nproc; grep -m1 'model name' /proc/cpuinfo; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-}"
       python3 -c "import os; print('affinity cores', len(os.sched_getaffinity(0)))"
       echo "cgroup cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo none)"
       (go version || echo "no go") 2>&1
       amd-smi static --clock 2>/dev/null | head -40) > "$OUT/info.txt" 2>&1
      ;;
    build)
      make -C "$ROOT" -j16 all > "$OUT/build.log" 2>&1 || { echo "build failed"; exit 1; }
      ;;
    tests)
      # the box's snapshot carries the built .so files but not build/*.o / *.s (.gpurunignore), so
      # check the libraries themselves against their sources rather than asking make
      for f in "$ROOT/bitcoin-miner_amd/minehip/libminehip.so" "$ROOT/oracle/liboracle_sha256.so"; do
        [ -f "$f" ] || { echo "missing $f: build first (make all)" | tee -a "$OUT/session.log"; exit 1; }
      done
      newer=$(find "$ROOT/bitcoin-miner_amd/csrc" "$ROOT/include" -newer "$ROOT/bitcoin-miner_amd/minehip/libminehip.so" \
              \( -name '*.hip' -o -name '*.cpp' -o -name '*.hpp' -o -name '*.h' -o -name '*.py' \) | head -3)
      [ -z "$newer" ] || echo "WARNING: sources newer than libminehip.so: $newer" | tee -a "$OUT/session.log"
      timeout -k 10 900 python -u -m pytest "$ROOT/tests" -m gpu -v -x -p no:cacheprovider --durations=25 --timeout 150 \
          --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/session.log"; tail -3 "$OUT/pytest_gpu.log"; fatal $rc
      ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/session.log"; fatal $rc
      ;;
    bench)
      # the driver's command line (BENCH_rNN.json)
      timeout -k 10 600 python "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; echo "bench rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/bench.json"; fatal $rc
      ;;
    multi1)
      # N = 1 through the in-process multi-device path (mh_search_multi, scheduler chunks)
      timeout -k 10 600 python "$ROOT/bench.py" --gpus 1 --multi --steps 20 --warmup 5 --no-pmc --no-cpu-baseline \
          > "$OUT/bench_multi1.json" 2> "$OUT/bench_multi1.err"
      rc=$?; echo "multi1 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/bench_multi1.json"; fatal $rc
      # the scheduler path itself: 4 worker threads on the one GPU, configs[3] slices (2^38 to stay short)
      timeout -k 10 600 python "$ROOT/bench.py" --gpus 4 --devices 0,0,0,0 --bits 38 --steps 8 --warmup 1 \
          > "$OUT/bench_multi4.json" 2> "$OUT/bench_multi4.err"
      rc=$?; echo "multi4 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/bench_multi4.json"; fatal $rc
      timeout -k 10 600 python "$ROOT/bench.py" --gpus 1 --config 4 --bits 38 --steps 8 --warmup 1 --no-pmc \
          --no-cpu-baseline > "$OUT/bench_single38.json" 2> "$OUT/bench_single38.err"
      rc=$?; echo "single38 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/bench_single38.json"; fatal $rc
      ;;
    cfg4)
      # configs[3] (2^40, the scaling workload) on one GPU: 20 slices covering the whole range
      timeout -k 10 600 python "$ROOT/bench.py" --gpus 1 --config 4 --steps 20 --warmup 1 --no-cpu-baseline \
          > "$OUT/bench_cfg4.json" 2> "$OUT/bench_cfg4.err"
      rc=$?; echo "cfg4 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/bench_cfg4.json"; fatal $rc
      ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
          -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-clock --no-n1 > "$OUT/prof_bench.json" 2> "$OUT/prof.err")
      rc=$?; echo "prof rc=$rc" | tee -a "$OUT/session.log"; fatal $rc
      find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \; | head -20
      # the per-(kernel, queue) summary that recomputes roofline.frac (tools/trace_frac.py)
      tr=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
      python3 "$ROOT/tools/trace_frac.py" "$OUT/prof_bench.json" "$tr" --stats-out "$OUT/kernel_stats_by_queue.csv" \
          > "$OUT/trace_frac.json" 2>&1; cat "$OUT/trace_frac.json"
      ;;
    inproc)
      # the in-process N-GPU path (mh_search_multi) modelled on this GPU: round-3 scheduler chain
      # against round-4 shards, configs[3] steps at N = 2, 4, 8 (tools/inproc_model.py)
      timeout -k 10 600 python "$ROOT/tools/inproc_model.py" --out "$OUT/inproc_model.json" > "$OUT/inproc.log" 2>&1
      rc=$?; echo "inproc rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/inproc.log"; fatal $rc
      ;;
    strong)
      # the launched N-GPU strong line (configs[3]) predicted on this GPU: every (step, rank) shard
      # timed alone, step time = the slowest rank's (tools/strong_shards.py)
      timeout -k 10 900 python "$ROOT/tools/strong_shards.py" --out "$OUT/strong_shards.json" > "$OUT/strong.log" 2>&1
      rc=$?; echo "strong rc=$rc" | tee -a "$OUT/session.log"; tail -5 "$OUT/strong.log"; fatal $rc
      ;;
    pmc)
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
          -d "$OUT/pmc1" -o run --output-format csv \
          -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --no-clock > /dev/null 2> "$OUT/pmc1.err")
      rc=$?; echo "pmc1 rc=$rc" | tee -a "$OUT/session.log"; fatal $rc
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace \
          -d "$OUT/pmc2" -o run --output-format csv \
          -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --no-clock > /dev/null 2> "$OUT/pmc2.err")
      rc=$?; echo "pmc2 rc=$rc" | tee -a "$OUT/session.log"; fatal $rc
      (cd /tmp && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace \
          -d "$OUT/pmc3" -o run --output-format csv \
          -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-pmc --no-clock > /dev/null 2> "$OUT/pmc3.err")
      rc=$?; echo "pmc3 rc=$rc" | tee -a "$OUT/session.log"; fatal $rc
      ;;
    listpmc)
      (cd /tmp && timeout -k 10 120 rocprofv3 -L > "$OUT/pmc_list.txt" 2>&1)
      rc=$?; echo "listpmc rc=$rc" | tee -a "$OUT/session.log"; grep -c . "$OUT/pmc_list.txt"; fatal $rc
      ;;
    valu)
      timeout -k 10 120 "$ROOT/build/valu_peak" > "$OUT/valu_peak.json" 2>&1
      rc=$?; echo "valu rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/valu_peak.json"; fatal $rc
      ;;
    valuops)
      timeout -k 10 300 "$ROOT/build/valu_ops" > "$OUT/valu_ops.json" 2>&1
      rc=$?; echo "valuops rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/valu_ops.json"; fatal $rc
      ;;
    valumix)
      timeout -k 10 300 "$ROOT/build/valu_mix" > "$OUT/valu_mix.json" 2>&1
      rc=$?; echo "valumix rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/valu_mix.json"; fatal $rc
      ;;
    valupair)
      timeout -k 10 300 "$ROOT/build/valu_pair" > "$OUT/valu_pair.json" 2>&1
      rc=$?; echo "valupair rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/valu_pair.json"; fatal $rc
      ;;
    valubank)
      timeout -k 10 300 "$ROOT/build/valu_bank" > "$OUT/valu_bank.json" 2>&1
      rc=$?; echo "valubank rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/valu_bank.json"; fatal $rc
      ;;
    kbench)
      timeout -k 10 600 python "$ROOT/tools/kbench.py" ${KBENCH_ARGS:-} > "$OUT/kbench.json" 2> "$OUT/kbench.err"
      rc=$?; echo "kbench rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/kbench.json"; tail -3 "$OUT/kbench.err"; fatal $rc
      ;;
    benchcfg)
      for c in 3a 3b; do
        timeout -k 10 600 python "$ROOT/bench.py" --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > "$OUT/bench_cfg$c.json" 2> "$OUT/bench_cfg$c.err"
        rc=$?; echo "bench cfg $c rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/bench_cfg$c.json"; fatal $rc
      done
      ;;
    latency)
      timeout -k 10 300 python "$ROOT/tools/latency.py" > "$OUT/latency.json" 2> "$OUT/latency.err"
      rc=$?; echo "latency rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/latency.json"; fatal $rc
      ;;
    cluster)
      timeout -k 10 300 python "$ROOT/tools/cluster_bench.py" --bits 36 --miners 4 > "$OUT/cluster.json" 2> "$OUT/cluster.err"
      rc=$?; echo "cluster rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/cluster.json"; fatal $rc
      timeout -k 10 300 python "$ROOT/tools/cluster_bench.py" --bits 36 --miners 4 --lose > "$OUT/cluster_lose.json" 2> "$OUT/cluster_lose.err"
      rc=$?; echo "cluster lose rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/cluster_lose.json"; fatal $rc
      ;;
    lspcluster)
      timeout -k 10 300 python "$ROOT/tools/lsp_cluster_bench.py" --bits 38 --miners 1 > "$OUT/lsp_cluster.json" 2> "$OUT/lsp_cluster.err"
      rc=$?; echo "lspcluster rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/lsp_cluster.json"; fatal $rc
      timeout -k 10 300 python "$ROOT/tools/lsp_cluster_bench.py" --bits 38 --miners 2 --kill 2 > "$OUT/lsp_cluster_kill.json" 2> "$OUT/lsp_cluster_kill.err"
      rc=$?; echo "lspcluster kill rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/lsp_cluster_kill.json"; fatal $rc
      ;;
    lspcfg4)
      # BASELINE configs[4] at its stated size on one GPU: server + 3 GPU miner processes + client
      # over LSP/UDP, 2^42 nonces, one miner SIGKILLed after 5 s; checked against a direct search
      # (LSP_MINERS=8: the configs[4] process layout, eight miner processes, all on the box's one GPU)
      timeout -k 10 900 python "$ROOT/tools/lsp_cluster_bench.py" --bits 42 --miners ${LSP_MINERS:-3} --kill 5 \
          > "$OUT/lsp_cfg4.json" 2> "$OUT/lsp_cfg4.err"
      rc=$?; echo "lspcfg4 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/lsp_cfg4.json"; fatal $rc
      ;;
    dist2)
      # 2 ranks on the box's one GPU: bench.py's launched path (configs[3] layout, 2^36 to stay short)
      BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29533 "$ROOT/bench.py" --gpus 2 --steps 4 --warmup 1 \
          --bits 36 > "$OUT/dist2.json" 2> "$OUT/dist2.err"
      rc=$?; echo "dist2 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/dist2.json"; fatal $rc
      # the same with one GPU visible per rank (a launcher isolating ranks): LOCAL_RANK 1 runs on
      # its only visible device, and the line says two ranks shared it
      HIP_VISIBLE_DEVICES=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29536 "$ROOT/bench.py" --gpus 2 --steps 4 --warmup 1 \
          --bits 36 > "$OUT/dist2_vis.json" 2> "$OUT/dist2_vis.err"
      rc=$?; echo "dist2 per-rank visibility rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/dist2_vis.json"; fatal $rc
      ;;
    dist8)
      # 8 ranks on the box's one GPU: bench.py's N = 8 sharding and host merge (2^36, golden-checked weak line too)
      BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
          --master-addr 127.0.0.1 --master-port 29534 "$ROOT/bench.py" --gpus 8 --steps 4 --warmup 1 \
          --bits 36 > "$OUT/dist8.json" 2> "$OUT/dist8.err"
      rc=$?; echo "dist8 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/dist8.json"; fatal $rc
      BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
          --master-addr 127.0.0.1 --master-port 29535 "$ROOT/bench.py" --gpus 8 --config 2 --bits 28 --steps 2 \
          --warmup 1 > "$OUT/dist8_weak.json" 2> "$OUT/dist8_weak.err"
      rc=$?; echo "dist8 weak rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/dist8_weak.json"; fatal $rc
      ;;
    rehearse8)
      # the N = 8 configs[3] lines end to end on the box's one GPU (all 8 workers / ranks share it, so
      # value and per_gpu_efficiency mean nothing here; the point is the whole path and golden_ok):
      # the in-process path (mh_search_multi over 8 listed devices) and the launched path (8 ranks)
      timeout -k 10 600 python "$ROOT/bench.py" --gpus 8 --devices 0,0,0,0,0,0,0,0 --steps 20 --warmup 2 \
          --no-clock > "$OUT/inproc8_cfg4.json" 2> "$OUT/inproc8_cfg4.err"
      rc=$?; echo "inproc8 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/inproc8_cfg4.json"; fatal $rc
      BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
          --master-addr 127.0.0.1 --master-port 29541 "$ROOT/bench.py" --gpus 8 --steps 20 --warmup 2 \
          --no-clock > "$OUT/dist8_cfg4.json" 2> "$OUT/dist8_cfg4.err"
      rc=$?; echo "dist8 cfg4 rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/dist8_cfg4.json"; fatal $rc
      ;;
    earlypmc)
      # round 5: configs[2]'s 60 x 'x' line with the Early layout (default) and without, PMC passes
      # included: VALU per nonce, issue per quad-cycle and waves per SIMD of each dominant kernel
      for e in 1 0; do
        MINEHIP_EARLY=$e timeout -k 10 600 python "$ROOT/bench.py" --config 3b --steps 5 --warmup 2 --no-cpu-baseline \
            > "$OUT/bench_cfg3b_early$e.json" 2> "$OUT/bench_cfg3b_early$e.err"
        rc=$?; echo "earlypmc $e rc=$rc" | tee -a "$OUT/session.log"; fatal $rc
      done
      ;;
    energy)
      # VALU instruction classes priced in joules at the power limit + the product's energy window
      # (tools/energy_probe.py, build/libvaluenergy.so)
      timeout -k 10 400 python "$ROOT/tools/energy_probe.py" --tag "$TAG" > "$OUT/energy_probe.log" 2>&1
      rc=$?; echo "energy rc=$rc" | tee -a "$OUT/session.log"; tail -14 "$OUT/energy_probe.log"; fatal $rc
      ;;
    layouts)
      # five fast_search layouts at the power limit: clock, W, J per 10^9 nonces (tools/energy_layouts.py)
      timeout -k 10 400 python "$ROOT/tools/energy_layouts.py" --tag "$TAG" > "$OUT/energy_layouts.log" 2>&1
      rc=$?; echo "layouts rc=$rc" | tee -a "$OUT/session.log"; tail -6 "$OUT/energy_layouts.log"; fatal $rc
      ;;
    ab:*)
      # an A/B recipe (tools/ab.py, tools/ab/<recipe>.json): one kbench process per workload
      recipe=${s#ab:}
      timeout -k 10 1500 python "$ROOT/tools/ab.py" "$ROOT/tools/ab/$recipe.json" --tag "$TAG/ab_$recipe" \
          > "$OUT/ab_$recipe.log" 2>&1
      rc=$?; echo "ab $recipe rc=$rc" | tee -a "$OUT/session.log"; cat "$OUT/ab_$recipe.log"; fatal $rc
      ;;
    *) echo "unknown step $s";;
  esac
done
echo "== done $(date +%T)" | tee -a "$OUT/session.log"
