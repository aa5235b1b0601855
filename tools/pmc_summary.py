"""Summarise a rocprofv3 PMC session of `bench.py --steps 1 --warmup 0
--no-cpu-baseline` (tools/gpu_session.sh step `pmc`) per kernel:

  VALU instructions per nonce   SQ_INSTS_VALU x 64 / nonces   (cross-check of nonce_ops)
  effective clock (GHz)         GRBM_GUI_ACTIVE / 8 XCDs / kernel time
  HBM bytes per launch          FETCH_SIZE x 2 (gfx950 wide-read correction) + WRITE_SIZE, x 1024
                                (MI355X_MICROARCH.md §HBM; separate --pmc passes)

Nonces per dispatch come from the host-only launch plan of the same search,
so this runs anywhere:  python tools/pmc_summary.py gpurun_out/<tag> [msg] [bits]
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]


def counters(path):
    per = defaultdict(dict)  # dispatch id -> {counter: value, name, dur}
    for r in csv.DictReader(open(path)):
        d = per[int(r["Dispatch_Id"])]
        d["name"] = r["Kernel_Name"]
        d["dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def main():
    base = sys.argv[1]
    msg = sys.argv[2] if len(sys.argv) > 2 else "cmu440"
    bits = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    import minehip
    fast = [p for p in minehip.plan(msg, 0, (1 << bits) - 1) if p["kind"] == 0]
    runs = {}
    for sub in ("pmc1", "pmc2", "pmc3"):
        f = os.path.join(base, sub, "run_counter_collection.csv")
        if os.path.exists(f):
            runs[sub] = counters(f)
    out = {}
    for sub, per in runs.items():
        disp = [per[k] for k in sorted(per) if "fast_search" in per[k]["name"]]
        if len(disp) != len(fast):
            raise SystemExit(f"{sub}: {len(disp)} fast dispatches but the plan has {len(fast)}")
        for d, p in zip(disp, fast):
            name = d["name"].split("(")[0]
            o = out.setdefault(name, {"dispatches": 0, "nonces": 0, "ns": 0, "nonce_ops": p["nonce_ops"]})
            if sub == "pmc1":
                o["dispatches"] += 1
                o["nonces"] += p["count"]
                o["ns"] += d["dur"]
                o["SQ_INSTS_VALU"] = o.get("SQ_INSTS_VALU", 0) + d.get("SQ_INSTS_VALU", 0)
                o["GRBM_GUI_ACTIVE"] = o.get("GRBM_GUI_ACTIVE", 0) + d.get("GRBM_GUI_ACTIVE", 0)
            for c in ("FETCH_SIZE", "WRITE_SIZE"):
                if c in d:
                    o[c] = o.get(c, 0) + d[c]
    for name, o in out.items():
        if o.get("nonces"):
            o["valu_instr_per_nonce"] = round(o["SQ_INSTS_VALU"] * 64 / o["nonces"], 1)
            o["ghz_effective"] = round(o["GRBM_GUI_ACTIVE"] / 8 / o["ns"], 3)
            o["ghs"] = round(o["nonces"] / o["ns"], 3)
        if "FETCH_SIZE" in o and "WRITE_SIZE" in o and o["dispatches"]:
            o["hbm_bytes_per_launch"] = int((2 * o["FETCH_SIZE"] + o["WRITE_SIZE"]) * 1024 / o["dispatches"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
