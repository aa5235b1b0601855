"""Extra rocprofv3 --pmc passes over one launch of the dominant configs[1]
kernel (fast_search<4,0>), e.g. the instruction-cache counters behind
DESIGN.md §4's issue-rate analysis.  One pass per counter set, each run under
bench.py's pmc_counters (separate rocprofv3 runs, block limits respected).

  python tools/pmc_extra.py [icache|valu] > gpurun_out/<tag>/pmc_extra.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]

SETS = {
    # one SQC counter per pass: the SQC block's per-pass limit is not in the guide
    "icache": (("GRBM_GUI_ACTIVE", "SQ_IFETCH", "SQ_IFETCH_LEVEL", "SQC_ICACHE_REQ"),
               ("GRBM_GUI_ACTIVE", "SQC_ICACHE_BUSY_CYCLES"),
               ("GRBM_GUI_ACTIVE", "SQC_ICACHE_MISSES"),
               ("GRBM_GUI_ACTIVE", "SQC_ICACHE_HITS")),
    "valu": (("GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VALU2",
              "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "SQ_BUSY_CYCLES"),),
}


def main():
    import bench
    import minehip  # noqa: F401
    which = sys.argv[1] if len(sys.argv) > 1 else "icache"
    msg = "cmu440"
    piece = bench.largest_piece(msg.encode(), 0, (1 << 32) - 1, {"word": 4, "mode": 0})
    vals, err = bench.pmc_counters(msg, [piece], 0, passes=SETS[which])
    if vals is None:
        print(json.dumps({"error": err}))
        sys.exit(1)
    v = next(iter(vals.values()))
    out = {"kernel": "fast_search<4, 0>", "nonces": piece["count"], "counters": v}
    for i in range(len(SETS[which])):
        g, d = v.get(f"GRBM_GUI_ACTIVE@{i}"), v.get(f"dur_ns@{i}")
        if g and d:
            out[f"cycles@{i}"] = g / 8
            out[f"sclk_ghz@{i}"] = round(g / 8 / d, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
