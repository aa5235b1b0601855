"""Predict bench.py's N-GPU strong-scaling line (BASELINE configs[3]: "cmu440",
[0, 2^40-1]) on ONE GPU.

At N GPUs the driver's launched bench runs K = 20 timed steps; in step k rank r
searches bench.rank_range(CONFIGS["4"], r, N, k, 20) on its own device and every
step ends in a host merge (gloo all_gather) that waits for the slowest rank.
This tool runs every (k, r) shard in turn on device 0, one mh_search (one sync)
each, and predicts the N-GPU wall time as sum_k max_r t(k, r): each GPU is
assumed to run its shard as fast as this GPU runs it alone (no cross-device
clock spread, no gloo cost).  Per-GPU efficiency = predicted GH/s / (N x the
N = 1 sequence's GH/s).

  python tools/strong_shards.py --out gpurun_out/strong.json [--ns 1,2,4,8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]
import bench  # noqa: E402  (rank_range, CONFIGS: the exact shards the bench runs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="4")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    torch.cuda.device_count()
    import minehip
    cfg = bench.CONFIGS[a.config]
    msg = cfg["msg"].encode()
    minehip.search(msg, 10 ** 12, 10 ** 12 + (1 << 30))  # warm up (module load, clocks)
    out = {"config": a.config, "steps": a.steps, "by_n": {}}
    base = None
    for n in [int(x) for x in a.ns.split(",")]:
        t_steps, per = [], []
        best = None
        for k in range(a.steps):
            ts = []
            for r in range(n):
                lo, hi = bench.rank_range(cfg, r, n, k, a.steps)
                t0 = time.perf_counter()
                res = minehip.search(msg, lo, hi)
                ts.append(time.perf_counter() - t0)
                best = res if best is None else min(best, res)
            t_steps.append(max(ts))
            per.append([round(x * 1e3, 3) for x in ts])
            print(f"N={n} step {k}: max {max(ts) * 1e3:.2f} ms min {min(ts) * 1e3:.2f} ms", flush=True)
        total = (1 << cfg["bits"]) if cfg["scaling"] == "strong" else (1 << cfg["bits"]) * n * a.steps
        busy = sum(sum(p) for p in per) / 1e3  # GPU-seconds of work over all ranks
        pred = total / sum(t_steps) / 1e9
        row = {"pred_ghs": round(pred, 4), "pred_s": round(sum(t_steps), 4),
               "gpu_seconds": round(busy, 4), "per_gpu_ghs_if_no_wait": round(total / busy / 1e9 * 1, 4),
               "result": list(best), "step_ms": per}
        if n == 1:
            base = pred
        if base:
            row["per_gpu_eff_vs_n1"] = round(pred / (n * base), 4)
            # the two loss terms: shard work slower than the N = 1 slices (tails), and waiting for
            # the slowest rank of each step (imbalance)
            row["work_eff"] = round(total / busy / 1e9 / base, 4)
            row["balance_eff"] = round(busy / (n * sum(t_steps)), 4)
        out["by_n"][str(n)] = row
        print(json.dumps({k: v for k, v in row.items() if k != "step_ms"} | {"n": n}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
