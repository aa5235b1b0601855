"""Recompute bench.py's roofline.frac from a rocprofv3 kernel trace of the same command.

  python tools/trace_frac.py <bench line .json> <run_kernel_trace.csv>

The trace names every lane length of a variant alike (`mh::fast_search<J, MODE>`), so the
dominant launches are told apart by grid size: the bench line's nonces_per_launch / 10^L runs,
rounded up to 256-lane workgroups.  Work-queue launches (MINEHIP_QUEUE=1, the default since
round 3) all have the resident grid, so there they are told apart by hardware queue instead: the
dominant (full-L) pieces run on the high-priority stream, whose dispatches of the kernel are the
long ones.  frac = alg_instr_per_nonce x nonces_per_launch / the trace's average
duration of those dispatches / peak.
"""
import csv
import json
import sys


def main():
    line = json.loads(open(sys.argv[1]).read())
    r = line["roofline"]
    L = r.get("lo_digits") or 3
    runs = r["nonces_per_launch"] // 10 ** L
    grid = -(-runs // 256) * 256
    name = r["kernel"].replace("mh::", "")
    rows = [x for x in csv.DictReader(open(sys.argv[2])) if name in x["Kernel_Name"]]

    def dur(x):
        return (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) * 1e-9

    durs = [dur(x) for x in rows if int(x["Grid_Size_X"]) == grid]
    match = f"grid {grid}"
    if not durs:  # work-queue launches: the queue whose dispatches of this kernel are longest
        by_q = {}
        for x in rows:
            by_q.setdefault(x["Queue_Id"], []).append(dur(x))
        if by_q:
            q, durs = max(by_q.items(), key=lambda kv: sum(kv[1]) / len(kv[1]))
            match = f"queue {q} (work queue)"
    if not durs:
        sys.exit(f"no {name} dispatch in the trace")
    avg = sum(durs) / len(durs)
    frac = r["alg_instr_per_nonce"] * r["nonces_per_launch"] / avg / 1e12 / r["peak"]
    out = {"kernel": r["kernel"], "lo_digits": L, "matched": match, "dispatches": len(durs),
           "trace_avg_ms": round(avg * 1e3, 4), "bench_avg_ms": r["avg_launch_ms"],
           "frac_from_trace": round(frac, 4), "frac_bench": r["frac"],
           "rel_diff": round(frac / r["frac"] - 1, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
