"""Recompute bench.py's roofline.frac from a rocprofv3 kernel trace of the same command.

  python tools/trace_frac.py <bench line .json> <run_kernel_trace.csv>

The trace names every lane length of a variant alike (`mh::fast_search<J, MODE>`), so the
dominant launches are told apart by grid size: the bench line's nonces_per_launch / 10^L runs,
rounded up to 256-lane workgroups.  frac = alg_instr_per_nonce x nonces_per_launch / the
trace's average duration of those dispatches / peak.
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
    durs = [(int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) * 1e-9
            for x in csv.DictReader(open(sys.argv[2]))
            if name in x["Kernel_Name"] and int(x["Grid_Size_X"]) == grid]
    if not durs:
        sys.exit(f"no {name} dispatch with grid {grid} in the trace")
    avg = sum(durs) / len(durs)
    frac = r["alg_instr_per_nonce"] * r["nonces_per_launch"] / avg / 1e12 / r["peak"]
    out = {"kernel": r["kernel"], "lo_digits": L, "grid": grid, "dispatches": len(durs),
           "trace_avg_ms": round(avg * 1e3, 4), "bench_avg_ms": r["avg_launch_ms"],
           "frac_from_trace": round(frac, 4), "frac_bench": r["frac"],
           "rel_diff": round(frac / r["frac"] - 1, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
