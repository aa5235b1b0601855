"""Recompute bench.py's roofline.frac from a rocprofv3 kernel trace of the same command, and write
the per-(kernel, queue) summary the recomputation uses.

  python tools/trace_frac.py <bench line .json> <run_kernel_trace.csv> [--stats-out <csv>]

rocprofv3's own --stats summary has one row per kernel name, and the trace names every lane length
of a variant alike (`mh::fast_search<J, MODE>`): configs[1]'s row for fast_search<4, 0> averages
the coarse L = 3 launches (~57 ms) with the L = 2 tail-split launches of the same kernel (~5 ms),
so frac cannot be recomputed from it.  The launches are told apart here:

* by grid size when launches are one workgroup per chunk (MINEHIP_QUEUE=0): the bench line's
  nonces_per_launch / 10^L runs, rounded up to 256-lane workgroups;
* by hardware queue with work-queue launches (the default; every launch has the resident grid):
  the coarse (full-L) pieces run on the high-priority stream, the others on the low-priority one
  (DESIGN.md §3), so the dominant kernel's queue with the longest average dispatch is the coarse
  one.

--stats-out writes one row per (kernel, queue) -- calls, total / average / min / max ns -- with the
coarse queue of the dominant kernel labelled with its lane length L; frac = alg_instr_per_nonce x
nonces_per_launch / that row's average / peak.  tests/test_bench_roofline.py
recomputes the committed line's frac from the committed summary.
"""
import argparse
import csv
import json


def dur_ns(x):
    return int(x["End_Timestamp"]) - int(x["Start_Timestamp"])


def by_queue_stats(rows, dominant=None, coarse_queue=None, lo_digits=None):
    """[(kernel, queue, role, L, calls, total, avg, min, max)] over the trace's dispatches."""
    acc = {}
    for x in rows:
        acc.setdefault((x["Kernel_Name"], x["Queue_Id"]), []).append(dur_ns(x))
    out = []
    for (name, q), ds in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        coarse = dominant is not None and dominant in name and q == coarse_queue
        role = "coarse (high-priority stream, full L)" if coarse else (
            "other pieces (low-priority stream)" if dominant is not None and dominant in name else "")
        out.append({"Name": name, "Queue_Id": q, "Role": role, "Lo_Digits": lo_digits if coarse else "",
                    "Calls": len(ds), "TotalDurationNs": sum(ds), "AverageNs": round(sum(ds) / len(ds), 2),
                    "MinNs": min(ds), "MaxNs": max(ds)})
    return out


def frac_from_stats(line, stats):
    """roofline.frac recomputed from the by-queue summary's coarse row of the dominant kernel."""
    r = line["roofline"]
    row = next(s for s in stats if s["Lo_Digits"] not in ("", None))
    avg = float(row["AverageNs"]) * 1e-9
    return r["alg_instr_per_nonce"] * r["nonces_per_launch"] / avg / 1e12 / r["peak"], row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("line")
    ap.add_argument("trace")
    ap.add_argument("--stats-out", default=None)
    a = ap.parse_args()
    line = json.loads(open(a.line).read())
    r = line["roofline"]
    L = r.get("lo_digits") or 3
    runs = r["nonces_per_launch"] // 10 ** L
    grid = -(-runs // 256) * 256
    name = r["kernel"].replace("mh::", "")
    all_rows = list(csv.DictReader(open(a.trace)))
    rows = [x for x in all_rows if name in x["Kernel_Name"]]

    durs = [dur_ns(x) * 1e-9 for x in rows if int(x["Grid_Size_X"]) == grid]
    match = f"grid {grid}"
    coarse_q = None
    if not durs:  # work-queue launches: the queue whose dispatches of this kernel are longest
        by_q = {}
        for x in rows:
            by_q.setdefault(x["Queue_Id"], []).append(dur_ns(x) * 1e-9)
        if by_q:
            coarse_q, durs = max(by_q.items(), key=lambda kv: sum(kv[1]) / len(kv[1]))
            match = f"queue {coarse_q} (work queue)"
    if not durs:
        raise SystemExit(f"no {name} dispatch in the trace")
    avg = sum(durs) / len(durs)
    frac = r["alg_instr_per_nonce"] * r["nonces_per_launch"] / avg / 1e12 / r["peak"]
    out = {"kernel": r["kernel"], "lo_digits": L, "matched": match, "dispatches": len(durs),
           "trace_avg_ms": round(avg * 1e3, 4), "bench_avg_ms": r["avg_launch_ms"],
           "frac_from_trace": round(frac, 4), "frac_bench": r["frac"],
           "rel_diff": round(frac / r["frac"] - 1, 4)}
    if a.stats_out:
        if coarse_q is None:  # grid-matched launches: label the queue they ran on
            coarse_q = next(x["Queue_Id"] for x in rows if int(x["Grid_Size_X"]) == grid)
        st = by_queue_stats(all_rows, name, coarse_q, L)
        with open(a.stats_out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0]))
            w.writeheader()
            w.writerows(st)
        out["stats_out"] = a.stats_out
        out["frac_from_stats"] = round(frac_from_stats(line, st)[0], 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
