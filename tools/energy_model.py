"""tools/energy_model.py -- the add3 split (and the other loop variants) priced under a fixed power
budget instead of the issue bound max(H, N/2).

The fast kernel runs at the firmware's package-power limit (PPT active for about half of every
window, `roofline.energy.limit_active_share`), so a variant's clock is set by how much power its
instruction stream draws per cycle, and its rate is clock / quad-cycles per nonce.  The model:

    P - P_floor = c * f^kappa * A,     A = (H + rho * F + sigma * S) / Q

  P        socket power at the limit (each variant's own mean W over its energy window)
  P_floor  the chip with every wave slot resident but idle (tools/valu_energy.hip "sleep")
  f        the kernel clock read inside the GPU during the same window (tools/clock_probe.hip)
  H, F, S  half-rate VALU, full-rate VALU and s_setprio instructions per 64 nonces (one wave
           iteration of the per-nonce loop, counted in the variant's assembly)
  Q        SIMD quad-cycles per 64 nonces, measured (kbench: clock / search rate)
  kappa    how power per unit of activity grows with the clock (f * V(f)^2: 1 + 2 * gamma when the
           voltage goes as f^gamma); rho, sigma the energy of a full-rate VALU instruction and of a
           marker against a half-rate one, inside the kernel's own mixed stream

kappa and rho are fitted on the variants of one A/B (same box, same process); sigma is taken from
the probes (a marker against an alignbit, each in a stream of its own).  The fixed-power rate of a
variant is then R = f / Q with f = ((P_cap - P_floor) / (c A))^(1/kappa): at a fixed budget a
variant wins by issuing its nonces in fewer quad-cycles only as far as the energy per quad-cycle
it adds does not cost more clock.  The same fit predicts round 3's split result (HISTORY.md §4:
none -> every third add3 split: quad-cycles 720 -> 675 per 64 nonces, clock -4.6%, rate +1.9% on
the d = 10 bucket) from round 3's quad-cycles alone, and ranks split counts the A/B did not build.

  python tools/energy_model.py --ab profiles/r06b_kbench_energy_split.json \\
      --probe profiles/r06a_energy_probe.json [--out profiles/r06b_energy_model.json]

Counting the loops needs the variants' assembly: `python tools/isa_variant.py prio a3split6 ...`
(build/isa/<variant>.s); the product build is build/fast_search_prio.s.
"""
import argparse
import collections
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd", "csrc"))

KERNEL = "_ZN2mh11fast_searchILi4ELi0EE"  # fast_search<4, One>: configs[1]'s d = 10 bucket
SIMDS = 1024


def loop_lines(body):
    """The instruction lines of the per-nonce loop (loop_mix.per_nonce_loop's block, operands kept)."""
    lines = body.split("\n")
    best, best_n = [], -1
    for i, l in enumerate(lines):
        if "Loop Header" not in l:
            continue
        block = []
        for j in range(i, len(lines)):
            t = lines[j].strip()
            if t and not t.startswith((";", ".")):
                block.append(t)
            if t.startswith("s_cbranch_scc") or t.startswith("s_branch"):
                break
        n = sum(x.startswith("v_") for x in block)
        if n > best_n:
            best, best_n = block, n
    return best


def op_key(line):
    """An instruction's opcode, with a v_bitop3's truth table (0x96 xor3, 0xca Ch, 0xe8 Maj)."""
    op = line.split()[0]
    if op.startswith("v_bitop3"):
        import re
        m = re.search(r"bitop3:(0x[0-9a-fA-F]+)", line)
        return f"{op}:{m.group(1).lower()}" if m else op
    return op


def loop_counts(s_path, kernel=KERNEL):
    """(H, F, S) of the kernel's per-nonce loop in an assembly file, plus the opcode histogram."""
    import loop_mix
    from valu_rates import valu_rate
    for name, body in loop_mix.kernels(open(s_path).read()).items():
        if name.startswith(kernel):
            ins = [op_key(x) for x in loop_lines(body) if x.startswith("v_") or x.startswith("s_setprio")]
            valu = [x for x in ins if x != "s_setprio"]
            h = sum(1 for x in valu if valu_rate(x.split(":")[0]) == "H")
            return {"H": h, "F": len(valu) - h, "S": ins.count("s_setprio"),
                    "ops": dict(collections.Counter(ins).most_common())}
    raise SystemExit(f"{kernel} not in {s_path}")


def variant_asm(name, recipe=None):
    """The assembly of an A/B variant: the product build, or the code object the recipe names."""
    if name == "product":
        return os.path.join(ROOT, "build", "fast_search_prio.s")
    co = (recipe or {}).get("code_objects", {}).get(name)
    if co:
        return os.path.join(ROOT, co[:-len(".hsaco")] + ".s")
    return os.path.join(ROOT, "build", "isa", f"{name}.s")


def probe_prices(probe):
    """pJ per wave-instruction of each probe class over the sleep floor, from an energy_probe.json
    (the median over its rounds), and the floor / idle watts."""
    rows = collections.defaultdict(list)
    for rnd in probe["rounds"]:
        for r in rnd:
            rows[r.get("kind")].append(r)

    def med(v):
        v = sorted(v)
        return v[len(v) // 2]

    floor = med([r["mean_w"] for r in rows["sleep"]])
    out = {"floor_w": floor, "idle_w": med([r["mean_w"] for r in rows["idle"]]) if rows["idle"] else None,
           "floor_clock_ghz": med([r["clock_ghz"] for r in rows["sleep"]]), "pj_per_wave_instr": {},
           "classes": {}}
    salu_pj = None
    for k in ["setprio"] + [k for k in rows if k != "setprio"]:
        rs = rows.get(k)
        if not rs or k in ("idle", "sleep") or not k or k.startswith("product"):
            continue
        w = med([r["mean_w"] for r in rs])
        nv = med([r.get("valu_wave_instr_per_s") or 0 for r in rs])
        ns = med([r.get("salu_wave_instr_per_s") or 0 for r in rs])
        out["classes"][k] = {"mean_w": w, "clock_ghz": med([r["clock_ghz"] for r in rs]),
                             "valu_per_simd_quad": med([r.get("valu_per_simd_quad") or 0 for r in rs]),
                             "ppt_share": med([(r.get("limit_active_share") or {}).get("ppt_pwr", 0) for r in rs])}
        if k == "setprio" and ns:
            salu_pj = (w - floor) / ns * 1e12
            out["pj_per_wave_instr"][k] = round(salu_pj, 1)
        elif nv:
            # a VALU probe's markers (h4f4_prio, h4b4_prio) at the markers' own price
            out["pj_per_wave_instr"][k] = round(((w - floor) - ns * (salu_pj or 0) * 1e-12) / nv * 1e12, 1)
    return out


# opcode -> probe class for the priced model (csrc/valu_rates.py's half-rate ops that are not
# rotations are priced as add3, the full-rate ones that are not bitop3 as add)
def price_class(op, prices=None):
    """The probe class an opcode (op_key) is priced at: its own probe where there is one (Ch, Maj
    and the shifts from round 6's second set), else its rate class's representative."""
    from valu_rates import valu_rate
    have = prices or {}
    if op == "s_setprio":
        return "setprio"
    if op.startswith("v_alignbit"):
        return "alignbit"
    if op.startswith("v_bitop3"):
        table = {"0xca": "bitop3_ch", "0xe8": "bitop3_maj"}.get(op.partition(":")[2])
        return table if table in have else "bitop3"
    if op.startswith("v_lshrrev_b32") and "lshr" in have:
        return "lshr"
    return "add3" if valu_rate(op.split(":")[0]) == "H" else "add"


def loop_energy(ops, pr):
    """pJ per 64 nonces of a loop (its opcode histogram) at the probes' prices."""
    pj = pr["pj_per_wave_instr"]
    return sum(n * pj[price_class(op, pj)] for op, n in ops.items())


def fit_priced(points, pr):
    """The priced model: A = loop_energy / Q from the probes' class prices (nothing about the
    variants' mix is fitted); least squares of ln(P - floor) = ln c + kappa ln f + ln A.
    Returns (rms, ln c, kappa)."""
    floor = pr["floor_w"]
    xs = [math.log(p["f"]) for p in points]
    ys = [math.log(p["P"] - floor) - math.log(loop_energy(p["ops"], pr) / p["Q"]) for p in points]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    kappa = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    lnc = my - kappa * mx
    return math.sqrt(sum((y - lnc - kappa * x) ** 2 for x, y in zip(xs, ys)) / n), lnc, kappa


def priced_clock(pm, pr, ops, Q, p_cap):
    """Clock (GHz) of a loop at the budget p_cap under the priced model pm."""
    A = loop_energy(ops, pr) / Q
    return math.exp((math.log(p_cap - pr["floor_w"]) - pm["ln_c"] - math.log(A)) / pm["kappa"])


def fit(points, sigma, floor):
    """Least squares of ln(P - floor) = ln c + kappa ln f + ln A(rho) over a grid of rho.
    points: [{"H", "F", "S", "Q", "f", "P"}].  Returns (rms, ln c, kappa, rho)."""
    best = None
    for i in range(1, 601):
        rho = i / 200  # 0.005 .. 3.0
        xs = [math.log(p["f"]) for p in points]
        ys = [math.log(p["P"] - floor) - math.log((p["H"] + rho * p["F"] + sigma * p["S"]) / p["Q"]) for p in points]
        n = len(xs)
        mx, my = sum(xs) / n, sum(ys) / n
        sxx = sum((x - mx) ** 2 for x in xs)
        if sxx <= 0:
            continue
        kappa = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx
        lnc = my - kappa * mx
        rms = math.sqrt(sum((y - lnc - kappa * x) ** 2 for x, y in zip(xs, ys)) / n)
        if kappa > 0 and (best is None or rms < best[0]):
            best = (rms, lnc, kappa, rho)
    return best


def predict(m, H, F, S, Q, p_cap):
    """Clock (GHz) and rate (GH/s) of a loop at the budget p_cap under model m."""
    A = (H + m["rho"] * F + m["sigma"] * S) / Q
    f = math.exp((math.log(p_cap - m["floor_w"]) - m["ln_c"] - math.log(A)) / m["kappa"])
    return f, f * 1e9 * SIMDS * 16 / Q / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ab", required=True, help="kbench JSON with --energy rounds per variant")
    ap.add_argument("--probe", required=True, help="energy_probe.json")
    ap.add_argument("--recipe", default=os.path.join(ROOT, "tools", "ab", "r06_energy_split.json"),
                    help="the A/B recipe (maps variant names to code objects)")
    ap.add_argument("--layouts", default=None,
                    help="tools/energy_layouts.py JSON: predict other loops' clocks (kappa from --ab, the scale "
                         "set on the one4 layout, prices from --probe)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ab = json.load(open(a.ab))
    recipe = json.load(open(a.recipe)) if a.recipe and os.path.exists(a.recipe) else None
    pr = probe_prices(json.load(open(a.probe)))
    pj = pr["pj_per_wave_instr"]
    sigma = pj.get("setprio", 0.0) / pj["alignbit"] if pj.get("alignbit") else 0.0
    points, skipped = {}, {}
    for name, v in ab.items():
        e = v.get("energy") or {}
        if not (e.get("ghz_med") and e.get("mean_w_med") and e.get("simd_quads_per_64_nonces")):
            skipped[name] = "no energy rounds"
            continue
        path = variant_asm(name, recipe)
        if not os.path.exists(path):
            skipped[name] = f"no assembly {os.path.relpath(path, ROOT)}"
            continue
        c = loop_counts(path)
        points[name] = dict(c, Q=e["simd_quads_per_64_nonces"], f=e["ghz_med"], P=e["mean_w_med"],
                            R=e["search_ghs_med"], j_per_gnonce=e.get("j_per_gnonce_med"),
                            wall_ghs_med=v.get("wall_ghs_med"), limiters=e.get("limiters"))
    # occupancy variants share the product's mix but not its register budget: fitted like the rest
    rms, lnc, kappa, rho = fit(list(points.values()), sigma, pr["floor_w"])
    m = {"ln_c": lnc, "kappa": kappa, "rho": rho, "sigma": sigma, "floor_w": pr["floor_w"], "rms_ln": rms}
    p_cap = sorted(p["P"] for p in points.values())[len(points) // 2]
    for p in points.values():
        f, R = predict(m, p["H"], p["F"], p["S"], p["Q"], p["P"])
        p["model_ghz"], p["model_ghs"] = round(f, 4), round(R, 3)

    # round 3's split A/B (HISTORY.md §4, profiles/r03n_*, r03o_*): quad-cycles per 64 nonces 720 / 675
    # at 2.301 / 2.196 GHz, the d = 10 bucket +1.9%; its loops had this build's mixes
    ns, sp = points.get("nosplit"), points.get("a3split3") or points.get("product")
    r3 = None
    if ns and sp:
        f0, R0 = predict(m, ns["H"], ns["F"], ns["S"], 720.0, p_cap)
        f1, R1 = predict(m, sp["H"], sp["F"], sp["S"], 675.0, p_cap)
        r3 = {"clock_change_pred": round(f1 / f0 - 1, 4), "clock_change_meas": round(2.196 / 2.301 - 1, 4),
              "rate_change_pred": round(R1 / R0 - 1, 4), "rate_change_meas_d10": 0.019,
              "rate_change_meas_range": [0.020, 0.026],
              "within_1pct": abs((R1 / R0 - 1) - 0.019) <= 0.01}

    # every split count s of the 201 add3 (continuous), Q from the issue bound with the pairing
    # efficiency interpolated between the built variants
    ranking = None
    if ns:
        built = sorted(((ns["H"] - p["H"], p) for n, p in points.items() if n != "split_w8" and p["F"] - ns["F"]
                        == 2 * (ns["H"] - p["H"])), key=lambda t: t[0])
        eff = [(s, max(p["H"], (p["H"] + p["F"]) / 2) / p["Q"]) for s, p in built]

        def eta(s):
            for (s0, e0), (s1, e1) in zip(eff, eff[1:]):
                if s0 <= s <= s1:
                    return e0 + (e1 - e0) * (s - s0) / (s1 - s0) if s1 > s0 else e0
            return eff[0][1] if s < eff[0][0] else eff[-1][1]

        def s_markers(s):
            for (s0, p0), (s1, p1) in zip(built, built[1:]):
                if s0 <= s <= s1:
                    return p0["S"] + (p1["S"] - p0["S"]) * (s - s0) / (s1 - s0) if s1 > s0 else p0["S"]
            return built[0][1]["S"] if s < built[0][0] else built[-1][1]["S"]

        rows = []
        for s in range(0, 202):  # the nosplit loop's 201 add3 (its H also holds the alignbits)
            H, F = ns["H"] - s, ns["F"] + 2 * s
            Q = max(H, (H + F) / 2) / eta(s)
            f, R = predict(m, H, F, s_markers(s), Q, p_cap)
            rows.append({"split": s, "H": H, "N": H + F, "S": round(s_markers(s), 1), "Q": round(Q, 1),
                         "ghz": round(f, 4), "ghs": round(R, 3)})
        top = max(rows, key=lambda r: r["ghs"])
        ranking = {"best": top, "every_third": next(r for r in rows if r["split"] == 67),
                   "issue_bound_best": min(rows, key=lambda r: max(r["H"], r["N"] / 2))["split"],
                   "all": rows}
    # the priced model: the probes' per-class prices set each loop's energy weight, only kappa and
    # the scale are fitted; round 3's split and the split counts the A/B did not build are predictions
    prm, plnc, pkap = fit_priced(list(points.values()), pr)
    pm = {"ln_c": plnc, "kappa": pkap, "rms_ln": prm}
    for p in points.values():
        f = priced_clock(pm, pr, p["ops"], p["Q"], p["P"])
        p["priced_ghz"], p["priced_ghs"] = round(f, 4), round(f * SIMDS * 16 / p["Q"], 3)
        p["loop_pj_per_64_nonces"] = round(loop_energy(p["ops"], pr))
    priced = {"model": pm, "round3_split": None, "split_ranking": None}
    if ns and sp:
        f0 = priced_clock(pm, pr, ns["ops"], 720.0, p_cap)
        f1 = priced_clock(pm, pr, sp["ops"], 675.0, p_cap)
        priced["round3_split"] = {
            "clock_change_pred": round(f1 / f0 - 1, 4), "clock_change_meas": round(2.196 / 2.301 - 1, 4),
            "rate_change_pred": round((f1 / 675.0) / (f0 / 720.0) - 1, 4), "rate_change_meas_d10": 0.019,
            "rate_change_meas_range": [0.020, 0.026],
            "within_1pct": abs((f1 / 675.0) / (f0 / 720.0) - 1 - 0.019) <= 0.01}
    if ranking:
        rows = []
        for r in ranking["all"]:
            s_ = r["split"]
            ops = dict(ns["ops"])
            ops["v_add3_u32"] = ops.get("v_add3_u32", 0) - s_
            ops["v_add_u32_e32"] = ops.get("v_add_u32_e32", 0) + 2 * s_
            ops["s_setprio"] = r["S"]
            f = priced_clock(pm, pr, ops, r["Q"], p_cap)
            rows.append({"split": s_, "Q": r["Q"], "ghz": round(f, 4), "ghs": round(f * SIMDS * 16 / r["Q"], 3)})
        priced["split_ranking"] = {"best": max(rows, key=lambda r: r["ghs"]),
                                   "every_third": next(r for r in rows if r["split"] == 67), "curve": rows[::6]}
    layouts = None
    if a.layouts:
        lay = json.load(open(a.layouts))
        asm = os.path.join(ROOT, "build", "fast_search_prio.s")
        rows = {}
        for name, v in lay.items():
            if not (v.get("ghz_med") and v.get("mean_w_med") and v.get("simd_quads_per_64_nonces")):
                continue
            c = loop_counts(asm, kernel=f"_ZN2mh11fast_searchILi{v['word']}ELi{v['mode']}EE")
            rows[name] = {"ops": c["ops"], "Q": v["simd_quads_per_64_nonces"], "f": v["ghz_med"],
                          "P": v["mean_w_med"], "j_per_gnonce": v.get("j_per_gnonce_med"),
                          "loop_pj_per_64_nonces": round(loop_energy(c["ops"], pr)), "valu": c["H"] + c["F"]}
        if "one4" in rows:
            ref = rows["one4"]
            # the scale on this box: ln c from the one4 layout at the fitted kappa
            lnc_box = (math.log(ref["P"] - pr["floor_w"]) - pkap * math.log(ref["f"])
                       - math.log(loop_energy(ref["ops"], pr) / ref["Q"]))
            pm_box = {"ln_c": lnc_box, "kappa": pkap}
            for name, r in rows.items():
                f = priced_clock(pm_box, pr, r["ops"], r["Q"], r["P"])
                r["ghz_pred"] = round(f, 4)
                r["err"] = round(f / r["f"] - 1, 4)
            layouts = {"kappa": round(pkap, 4), "scale_from": "one4", "rows": rows}
    if ranking:
        ranking["curve"] = ranking.pop("all")[::6]
    out = {"model": m, "p_cap_w": p_cap, "probe": pr, "points": points, "skipped": skipped, "priced": priced,
           "layouts": layouts,
           "round3_split": r3, "split_ranking": ranking,
           "note": "P - P_floor = c f^kappa (H + rho F + sigma S) / Q, fitted on one A/B's variants "
                   "(tools/energy_model.py)"}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s)
    print(s)


if __name__ == "__main__":
    main()
