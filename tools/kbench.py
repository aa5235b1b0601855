"""Kernel-level A/B bench: GH/s of the fast kernel on one decimal bucket
(HIP-event time from the library's profile counters), interleaving
configurations given as env settings inside ONE process.

  python tools/kbench.py --msg cmu440 --lo 1000000000 --count 2147483648 \
      --var base: --var lds3:MINEHIP_DEV_LDS=54000 --rounds 3

A --var that sets a MINEHIP_DEV_* hook needs the dev build of the library
(`make dev`); kbench then loads build/dev/libminehip.so for every variant, so
the A/B compares like with like.  The product library has no hooks.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# --pkg DIR: load the minehip package (and its libminehip.so) from DIR instead, e.g. an
# experimental build (build/<variant>/minehip); must come first on the command line
if len(sys.argv) > 2 and sys.argv[1] == "--pkg":
    sys.path[:0] = [sys.argv[2]]
    del sys.argv[1:3]
else:
    sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]
if any("MINEHIP_DEV_" in a for a in sys.argv) and not os.environ.get("MINEHIP_LIB"):
    os.environ["MINEHIP_LIB"] = os.path.join(ROOT, "build", "dev", "libminehip.so")
import minehip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msg", default="cmu440")
    ap.add_argument("--lo", type=int, default=10 ** 9)
    ap.add_argument("--count", type=int, default=1 << 31)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--var", action="append", default=[], help="name:K=V,K=V")
    ap.add_argument("--clock", action="store_true",
                    help="also read each variant's in-kernel clock during a 2^37-nonce search of "
                         "fast_search<4, One> (bench.kernel_clock; needs build/libclockprobe.so)")
    ap.add_argument("--energy", type=int, default=0, metavar="R",
                    help="R interleaved rounds of that clock search per variant, each also an energy "
                         "window (tools/energy.py: J per 10^9 nonces, mean W, the active limit)")
    a = ap.parse_args()
    variants = []
    for v in a.var or ["base:"]:
        name, _, kv = v.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        variants.append((name, env))
    res = {n: [] for n, _ in variants}
    minehip.search(a.msg, a.lo, a.lo + (1 << 26))  # warm up / load code objects
    for _ in range(a.rounds):
        for name, env in variants:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            minehip.profile_enable(0, True)
            t0 = time.perf_counter()
            r = minehip.search(a.msg, a.lo, a.lo + a.count - 1)
            wall = time.perf_counter() - t0
            p = minehip.profile_read(0)
            minehip.profile_enable(0, False)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            ns = p["fast_ns"] + p["generic_ns"]
            # ghs: over the sum of the launches' HIP-event times (meaningless when launches
            # overlap, MINEHIP_STREAMS=2); wall_ghs: over the search call's wall clock
            res[name].append({"ghs": a.count / ns, "fast_ghs": p["fast_nonces"] / max(1, p["fast_ns"]),
                              "wall_ghs": a.count / wall / 1e9, "result": r})
    out = {n: {"ghs_max": max(x["ghs"] for x in v), "ghs_med": sorted(x["ghs"] for x in v)[len(v) // 2],
               "wall_ghs_med": sorted(x["wall_ghs"] for x in v)[len(v) // 2],
               "wall_ghs_max": max(x["wall_ghs"] for x in v),
               "fast_ghs_max": max(x["fast_ghs"] for x in v), "result": v[-1]["result"]} for n, v in res.items()}
    if a.energy:
        sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
        import bench
        import energy
        meter = energy.meter_for_device(0)
        runs = {n: [] for n, _ in variants}
        for _ in range(a.energy):
            for name, env in variants:
                old = {k: os.environ.get(k) for k in env}
                os.environ.update(env)
                try:
                    kc = bench.kernel_clock(lambda m, lo, hi: minehip.search(m, lo, hi), 0, meter=meter)
                finally:
                    for k, v in old.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
                runs[name].append(kc or {})
        for name, rs in runs.items():
            def med(key, sub=None):
                v = [(r.get(sub) or {}).get(key) if sub else r.get(key) for r in rs]
                v = sorted(x for x in v if isinstance(x, (int, float)))
                return v[len(v) // 2] if v else None
            e = {"rounds": len(rs), "ghz_med": med("ghz"), "search_ghs_med": med("search_ghs"),
                 "j_per_gnonce_med": med("j_per_gnonce", "energy"), "mean_w_med": med("mean_w", "energy"),
                 "gfx_voltage_mv_med": med("gfx_voltage_mv", "energy"),
                 "limiters": sorted({(r.get("energy") or {}).get("limiter") or "?" for r in rs}),
                 "runs": [{"ghz": r.get("ghz"), "search_ghs": r.get("search_ghs"),
                           "ghz_by_xcd": r.get("ghz_by_xcd"), "energy": r.get("energy")} for r in rs]}
            if e["ghz_med"] and e["search_ghs_med"]:
                e["simd_quads_per_64_nonces"] = round(e["ghz_med"] / e["search_ghs_med"] * 1024 * 64 / 4, 1)
            out[name]["energy"] = e
    if a.clock:
        sys.path.insert(0, ROOT)
        import bench
        for name, env in variants:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            try:
                kc = bench.kernel_clock(lambda m, lo, hi: minehip.search(m, lo, hi))
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            out[name]["kernel_clock"] = kc
            if kc and kc.get("ghz"):
                # SIMD quad-cycles per 64 nonces (one wave-iteration of the loop) in the probed search,
                # at its own clock: 1,024 SIMDs, 4 cycles a quad; the <4, One> mix bound is 701
                out[name]["simd_quads_per_64_nonces"] = round(kc["ghz"] / kc["search_ghs"] * 1024 * 64 / 4, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
