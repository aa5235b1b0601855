"""tools/energy_layouts.py -- the clock, power and energy per nonce of other fast_search layouts, for
an out-of-sample check of tools/energy_model.py (round 6): its exponent was fitted on variants of
ONE loop (`<4, One>`'s add3 splits); here five different loops -- one- and two-block, last-digit and
Early -- each run alone at the power limit, and the model, with the probes' instruction prices and
one scale set on `<4, One>`, predicts the clock each of the others holds.

  python tools/energy_layouts.py --tag r06g [--rounds 3]

Per layout and round: an un-profiled search of one bucket (2^36-2^37 nonces, one dominant launch
layout) with the in-kernel clock probe (bench.kernel_clock) inside an energy window (tools/energy.py).
Writes gpurun_out/<tag>/energy_layouts.json.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd"), os.path.join(ROOT, "tools")]

# name -> (message, first nonce, nonces, the dominant layout (J, MODE) the planner gives the range)
LAYOUTS = {
    "one4": ("cmu440", 10 ** 11, 1 << 37, (4, 0)),                   # configs[1]'s d = 10 layout
    "one10": (("cmu440-" * 10)[:30], 10 ** 10, 1 << 36, (10, 0)),
    "one11": ("a" * 100, 10 ** 10, 1 << 36, (11, 0)),                 # configs[2]'s 100 x 'a'
    "preearly0": ("x" * 60, 10 ** 10, 1 << 36, (0, 4)),               # configs[2]'s 60 x 'x'
    "twoearly13": (("cmu440-" * 10)[:48], 10 ** 10, 1 << 36, (13, 5)),  # two blocks per nonce
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r06_layouts")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "gpurun_out", a.tag)
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, "energy_layouts.json")
    import torch
    torch.cuda.set_device(0)
    import bench
    import energy
    import minehip
    for name, (msg, lo, n, jm) in LAYOUTS.items():  # the plans really take these layouts
        top = max((p for p in minehip.plan(msg, lo, lo + n - 1) if p["kind"] == 0), key=lambda p: p["count"])
        assert (top["word"], top["mode"]) == jm, (name, top["word"], top["mode"])
    meter = energy.meter_for_device(0)
    if not meter.ok:
        raise SystemExit(f"energy counter not available: {meter.error}")
    minehip.search("cmu440", 10 ** 9, 10 ** 9 + (1 << 30))  # module load, clocks up
    runs = {k: [] for k in LAYOUTS}
    for _ in range(a.rounds):
        for name, (msg, lo, n, jm) in LAYOUTS.items():
            kc = bench.kernel_clock(lambda m, x, y: minehip.search(m, x, y), 0, delay_s=0.3, window_s=0.6,
                                    meter=meter, msg=msg, lo=lo, n=n)
            runs[name].append(kc or {})
            e = (kc or {}).get("energy") or {}
            print(json.dumps({"layout": name, "ghz": (kc or {}).get("ghz"), "ghs": (kc or {}).get("search_ghs"),
                              "w": e.get("mean_w"), "j_per_gnonce": e.get("j_per_gnonce")}), flush=True)

    def med(v):
        v = sorted(x for x in v if isinstance(x, (int, float)))
        return v[len(v) // 2] if v else None

    out = {}
    for name, rs in runs.items():
        msg, lo, n, jm = LAYOUTS[name]
        f = med([r.get("ghz") for r in rs])
        R = med([r.get("search_ghs") for r in rs])
        out[name] = {"msg_len": len(msg), "lo": lo, "nonces": n, "word": jm[0], "mode": jm[1],
                     "ghz_med": f, "search_ghs_med": R,
                     "mean_w_med": med([(r.get("energy") or {}).get("mean_w") for r in rs]),
                     "j_per_gnonce_med": med([(r.get("energy") or {}).get("j_per_gnonce") for r in rs]),
                     # SIMD quad-cycles per 64 nonces at the clock held (1,024 SIMDs, 4 cycles a quad)
                     "simd_quads_per_64_nonces": round(f / R * 1024 * 64 / 4, 1) if f and R else None,
                     "runs": rs}
    json.dump(out, open(path, "w"), indent=1)
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
