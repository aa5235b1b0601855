"""Predict the in-process N-GPU line (`python bench.py --gpus N`, mh_search_multi) on ONE GPU.

At N > 1 without a launcher, bench.py runs each configs[3] step ("cmu440", a 2^40/K slice) as one
mh_search_multi call over devices 0..N-1: one host thread per device.  Devices run independently,
so a step lasts as long as the busiest device's chain of searches.  This tool replays, on device
0, the exact chain each device would run and predicts the step time as the maximum over devices
of their summed search times (each timed search includes its plan, launches, drain and sync):

  old  the round-3 path: every call a fresh scheduler (mh_sched_*: 2^32 first chunk, 250 ms of
       the measured rate, capped at pending / 2N, >= 2^28), N miners on virtual clocks; each chunk
       it hands out is searched for real on device 0 and advances its miner's clock by that time.
  new  the round-4 path: mh_multi_plan's shards (equal weights: every device as fast as this one),
       one search per device, plus the dynamic tail (none at these sizes).

per-GPU efficiency = slice / predicted step time / (N x the slice's one-search rate on this GPU).

  python tools/inproc_model.py --out gpurun_out/inproc.json [--ns 2,4,8] [--steps 20]
"""
import argparse
import heapq
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]
import bench  # noqa: E402  (CONFIGS, step_range: the slices the bench runs)


def timed(minehip, msg, lo, hi):
    t0 = time.perf_counter_ns()
    r = minehip.search(msg, lo, hi)
    return r, time.perf_counter_ns() - t0


def old_path(minehip, msg, lo, hi, n):
    """The round-3 scheduler chain, replayed chunk by chunk on device 0."""
    s = minehip.Scheduler(init_chunk=1 << 32, min_chunk=1 << 28)
    for i in range(n):
        s.add_miner(i)
    s.submit(0, msg, lo, hi)
    clock = [(0, i) for i in range(n)]  # (virtual ns, miner): the next free miner asks first
    heapq.heapify(clock)
    chunks = [0] * n
    busy = [0] * n
    best = None
    done = None
    while done is None:
        t, i = heapq.heappop(clock)
        a = s.next(i, t)
        if a is None:  # nothing left for this miner: it idles until the job is done
            busy[i] = max(busy[i], t)
            continue
        _, _, clo, chi = a
        r, dt = timed(minehip, msg, clo, chi)
        best = r if best is None else min(best, r)
        chunks[i] += 1
        busy[i] = t + dt
        done = s.result(i, r[0], r[1], t + dt)
        heapq.heappush(clock, (t + dt, i))
    return {"step_ms": max(busy) / 1e6, "chunks_per_device": chunks, "result": list(best),
            "merged": list(done[2:])}


def new_path(minehip, msg, lo, hi, n):
    """The round-4 split: one head shard per device (+ tail chunks to the first free device)."""
    spans = minehip.multi_plan(msg, lo, hi, n)
    busy = [0] * n
    best = None
    for s in spans:
        if s["kind"] == 0:
            r, dt = timed(minehip, msg, s["lower"], s["upper"])
            busy[s["worker"]] += dt
            best = r if best is None else min(best, r)
    for s in spans:
        if s["kind"] == 1:
            i = min(range(n), key=lambda k: busy[k])
            r, dt = timed(minehip, msg, s["lower"], s["upper"])
            busy[i] += dt
            best = min(best, r)
    return {"step_ms": max(busy) / 1e6, "busy_ms": [round(b / 1e6, 3) for b in busy],
            "spans": len(spans), "result": list(best)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--slices", default=None, help="step indices to replay (default: 0 and K/2)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    torch.cuda.device_count()
    import minehip
    cfg = bench.CONFIGS["4"]
    msg = cfg["msg"].encode()
    minehip.search(msg, 10 ** 11, 10 ** 11 + (1 << 34))  # warm up (module load, clocks)
    ks = [int(x) for x in a.slices.split(",")] if a.slices else [0, a.steps // 2]
    out = {"config": "4", "steps": a.steps, "slices": {}}
    for k in ks:
        lo, hi = bench.step_range(cfg, k, a.steps)
        r1, t1 = timed(minehip, msg, lo, hi)
        base = (hi - lo + 1) / t1  # nonces per ns, one search on one GPU
        rows = {"range": [lo, hi], "n1_ms": round(t1 / 1e6, 3), "n1_ghs": round(base, 4), "by_n": {}}
        for n in [int(x) for x in a.ns.split(",")]:
            row = {}
            for name, fn in (("old", old_path), ("new", new_path)):
                m = fn(minehip, msg, lo, hi, n)
                assert m["result"] == list(r1), (name, n, m["result"], r1)
                m["pred_ghs"] = round((hi - lo + 1) / (m["step_ms"] * 1e6), 4)
                m["per_gpu_eff"] = round(m["pred_ghs"] / (n * base), 4)
                m["step_ms"] = round(m["step_ms"], 3)
                row[name] = m
                print(json.dumps({"slice": k, "n": n, "path": name,
                                  **{x: m[x] for x in ("step_ms", "pred_ghs", "per_gpu_eff")}}), flush=True)
            rows["by_n"][str(n)] = row
        out["slices"][str(k)] = rows
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
