"""Wall-clock latency of small searches (the request sizes a CPU-era server
hands a miner), median of repeated calls, plus the kernel-only time."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]
import minehip  # noqa: E402

out = {}
for msg, lo, hi in (("cmu440", 0, 9_999), ("cmu440", 0, 999_999), ("cmu440", 0, 9_999_999),
                    ("cmu440", 0, 99_999_999), ("x" * 60, 0, 9_999_999)):
    minehip.search(msg, lo, hi)
    ts = []
    for _ in range(20):
        t = time.perf_counter()
        minehip.search(msg, lo, hi)
        ts.append(time.perf_counter() - t)
    minehip.profile_enable(0, True)
    minehip.search(msg, lo, hi)
    p = minehip.profile_read(0)
    minehip.profile_enable(0, False)
    ts.sort()
    out[f"{msg[:8]}[{lo},{hi}]"] = {"median_ms": round(ts[len(ts) // 2] * 1e3, 4), "min_ms": round(ts[0] * 1e3, 4),
                                   "kernel_ms": round((p["fast_ns"] + p["generic_ns"]) / 1e6, 4),
                                   "pieces": len(minehip.plan(msg, lo, hi))}
print(json.dumps(out))
