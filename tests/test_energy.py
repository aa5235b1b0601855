"""The energy plumbing of the bench line and the fixed-power model, on CPU with stubs (VERDICT r05
items 1-2): tools/energy.py's window arithmetic and limiter choice, bench.energy_fields, the
per-device energy of the N > 1 paths (bench.kernel_clocks with meters), and tools/energy_model.py's
fit recovering known parameters."""
import math
import os
import sys

import pytest

from conftest import ROOT

sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
import bench  # noqa: E402
import energy  # noqa: E402
import energy_model  # noqa: E402


def _read(ns, joules, acc, ppt, thm=0):
    return {"host_ns": ns, "energy_j": joules, "energy_ts": ns,
            "viol": {"acc_counter": acc, "acc_ppt_pwr": ppt, "acc_socket_thrm": thm, "acc_vr_thrm": 0,
                     "acc_hbm_thrm": 0, "acc_prochot_thrm": 0, "acc_gfx_clk_below_host_limit": 0}}


def test_window_delta_energy_power_and_limiter():
    a, b = _read(0, 1000.0, 100, 10), _read(2_000_000_000, 3640.0, 300, 110)
    d = energy.window_delta(a, b, nonces=1 << 37)
    assert d["seconds"] == 2.0 and d["joules"] == 2640.0 and d["mean_w"] == 1320.0
    assert d["j_per_gnonce"] == round(2640.0 / ((1 << 37) / 1e9), 4)
    assert d["limit_active_share"]["ppt_pwr"] == 0.5 and d["limiter"] == "ppt_pwr"
    quiet = energy.window_delta(_read(0, 0.0, 0, 0), _read(10 ** 9, 400.0, 100, 1))
    assert quiet["limiter"] == "none reported" and "j_per_gnonce" not in quiet
    hot = energy.window_delta(_read(0, 0.0, 0, 0, 0), _read(10 ** 9, 400.0, 100, 0, 30))
    assert hot["limiter"] == "socket_thrm"
    bare = energy.window_delta({"host_ns": 0, "energy_error": "x"}, {"host_ns": 1})
    assert bare["energy_error"] == "x" and bare["limiter"] == "not exposed"


def test_parse_bdf():
    assert energy.parse_bdf("0000:75:00.0") == (0, 0x75, 0)
    assert energy.parse_bdf("0001:e5:1f.1\n") == (1, 0xE5, 0x1F)


class StubMeter:
    """A meter whose counters advance by `watts` per second of host time."""
    ok = True
    error = None

    def __init__(self, watts):
        self.watts = watts

    def read(self):
        import time
        t = time.perf_counter_ns()
        return _read(t, self.watts * t * 1e-9, t // 1000, t // 2000)

    def snapshot(self):
        return {"current_socket_power": self.watts, "power_limit_w": 1400.0, "gfx_clk_mhz": [2200] * 8}


def test_window_and_energy_fields():
    w = energy.Window(StubMeter(1300.0), nonces=10 ** 9, snap_after_s=0.01)
    import time
    with w:
        time.sleep(0.05)
    r = w.result
    assert abs(r["mean_w"] - 1300.0) < 1.0 and r["limiter"] == "ppt_pwr" and r["snapshot"]["power_limit_w"] == 1400.0
    f = bench.energy_fields(r, {"ghz": 2.2})
    assert f["kernel_clock_ghz"] == 2.2 and abs(f["j_per_gnonce"] - r["joules"]) < 1e-3
    assert f["power_limit_w"] == 1400.0 and f["limiter"] == "ppt_pwr"
    assert bench.energy_fields(None)["error"] and bench.energy_fields({"energy_error": "e"})["error"] == "e"
    # no meter at all: the Window still ends and says why
    w2 = energy.Window(None)
    with w2:
        pass
    assert w2.result["error"]


def test_kernel_clocks_pass_each_device_its_meter():
    """The in-process N > 1 line: one thread per device, each probe gets its own device's meter
    and returns its energy beside its clock (bench.py copies both into per_device)."""
    seen = {}

    def probe(search_dev, dev, meter=None):
        seen[dev] = meter
        return {"ghz": 2.0 + dev / 100, "energy": {"mean_w": meter.watts, "j_per_gnonce": 24.0 + dev}}

    meters = {d: StubMeter(1300.0 + d) for d in (0, 1, 3)}
    out = bench.kernel_clocks(lambda d: (lambda m, a, b: None), [0, 1, 1, 3], probe=probe, meters=meters)
    assert {d: seen[d].watts for d in seen} == {0: 1300.0, 1: 1301.0, 3: 1303.0}
    assert out[3]["energy"]["j_per_gnonce"] == 27.0 and out[1]["ghz"] == 2.01


def test_model_fit_recovers_known_parameters():
    """Points generated from P - floor = c f^kappa (H + rho F + sigma S) / Q are fitted back."""
    kappa, rho, sigma, lnc, floor = 2.6, 0.8, 0.03, math.log(0.05), 370.0
    pts = []
    for s, q in ((0, 720.0), (33, 700.0), (50, 690.0), (67, 675.0), (100, 680.0)):
        H, F, S = 703 - s, 493 + 2 * s, 400 + s // 3
        A = (H + rho * F + sigma * S) / q
        p_cap = 1320.0 + s * 0.05
        f = math.exp((math.log(p_cap - floor) - lnc - math.log(A)) / kappa)
        pts.append({"H": H, "F": F, "S": S, "Q": q, "f": f, "P": p_cap})
    rms, c, k, r = energy_model.fit(pts, sigma, floor)
    assert rms < 1e-3 and abs(k - kappa) < 0.05 and abs(r - rho) < 0.02
    m = {"ln_c": c, "kappa": k, "rho": r, "sigma": sigma, "floor_w": floor}
    f, R = energy_model.predict(m, pts[3]["H"], pts[3]["F"], pts[3]["S"], pts[3]["Q"], pts[3]["P"])
    assert abs(f / pts[3]["f"] - 1) < 2e-3 and abs(R - f * 16384 / pts[3]["Q"]) < 1e-9


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "build", "fast_search_prio.s")),
                    reason="needs the built assembly (make all)")
def test_loop_counts_of_the_product():
    """The product loop's classes as the model counts them: fast_search<4, One> per 64 nonces."""
    c = energy_model.loop_counts(os.path.join(ROOT, "build", "fast_search_prio.s"))
    assert c["H"] + c["F"] == 1263 and c["H"] == 636 and c["S"] > 0
    assert c["ops"]["v_alignbit_b32"] == 500 and c["ops"]["v_add3_u32"] == 134


def test_energy_total_over_devices():
    """The line's energy_timed: joules summed over devices, J per 10^9 nonces of all their nonces,
    the longest window for the mean power; ranks sharing a device (one-GPU rehearsals) flagged."""
    rows = [{"dev": 0, "nonces": 2 * 10 ** 9, "energy_timed": {"joules": 50.0, "seconds": 0.04}},
            {"dev": 1, "nonces": 2 * 10 ** 9, "energy_timed": {"joules": 52.0, "seconds": 0.05}},
            {"dev": 2, "nonces": 10 ** 9, "energy_timed": None}]
    t = bench.energy_total(rows)
    assert t["joules"] == 102.0 and t["j_per_gnonce"] == 25.5 and t["mean_w"] == 2040.0
    assert t["devices"] == 2 and t["shared_device"] is False
    rows[1]["dev"] = 0
    assert bench.energy_total(rows)["shared_device"] is True
    # launched ranks that each see one GPU all report device 0: their PCI addresses tell them apart
    rows[0]["pci"], rows[1]["pci"] = "0000:75:00", "0000:05:00"
    assert bench.energy_total(rows)["shared_device"] is False and bench.energy_total(rows)["devices"] == 2
    assert bench.energy_total([{"dev": 0, "nonces": 1, "energy_timed": {"energy_error": "x"}}]) is None


def test_priced_model_fit():
    """The priced model: loop energies from per-class prices, kappa and the scale fitted; points
    made with a known kappa are fitted back and each clock is reproduced."""
    pr = {"floor_w": 369.0, "pj_per_wave_instr": {"alignbit": 790.0, "add3": 990.0, "bitop3": 1120.0,
                                                  "add": 870.0, "setprio": 12.0}}
    base = {"v_alignbit_b32": 500, "v_bitop3_b32": 309, "v_lshrrev_b32_e32": 73, "s_setprio": 420}
    kappa, lnc = 2.4, -2.4
    pts = []
    for s, q in ((0, 765.0), (33, 729.0), (67, 700.0), (100, 707.0)):
        ops = dict(base, v_add3_u32=201 - s, v_add_u32_e32=111 + 2 * s)
        A = energy_model.loop_energy(ops, pr) / q
        f = math.exp((math.log(1334.0 - pr["floor_w"]) - lnc - math.log(A)) / kappa)
        pts.append({"ops": ops, "Q": q, "f": f, "P": 1334.0})
    rms, c, k = energy_model.fit_priced(pts, pr)
    assert rms < 1e-9 and abs(k - kappa) < 1e-6 and abs(c - lnc) < 1e-6
    pm = {"ln_c": c, "kappa": k}
    for p in pts:
        assert abs(energy_model.priced_clock(pm, pr, p["ops"], p["Q"], p["P"]) / p["f"] - 1) < 1e-9
    assert energy_model.price_class("v_xad_u32") == "add3" and energy_model.price_class("v_xor_b32_e32") == "add"


def test_committed_energy_model_reproduces_the_documented_numbers():
    """DESIGN §4 / HISTORY §4 quote the fixed-power model fitted on round 6's one-box data
    (profiles/r06g_energy_model.json: the variants' and layouts' loop histograms, quad-cycles,
    clocks and watts, and the probe prices).  Refitting from that file alone gives the quoted
    kappa, every variant's clock within 0.5%, round 3's split within 1% of its measured +1.9%,
    and the four other layouts' clocks within 2% (out of sample: the scale is set on <4, One>)."""
    import json
    d = json.load(open(os.path.join(ROOT, "profiles", "r06g_energy_model.json")))
    pr = d["probe"]
    pts = list(d["points"].values())
    rms, lnc, kap = energy_model.fit_priced(pts, pr)
    assert abs(kap - 2.26) < 0.01 and rms < 0.005
    pm = {"ln_c": lnc, "kappa": kap}
    for p in pts:
        assert abs(energy_model.priced_clock(pm, pr, p["ops"], p["Q"], p["P"]) / p["f"] - 1) < 0.005
    ns, sp, cap = d["points"]["nosplit"], d["points"]["a3split3"], d["p_cap_w"]
    f0 = energy_model.priced_clock(pm, pr, ns["ops"], 720.0, cap)
    f1 = energy_model.priced_clock(pm, pr, sp["ops"], 675.0, cap)
    assert abs((f1 / 675.0) / (f0 / 720.0) - 1 - 0.019) < 0.01 and abs(f1 / f0 - 1 + 0.0456) < 0.01
    rows = d["layouts"]["rows"]
    ref = rows["one4"]
    lnc_box = (math.log(ref["P"] - pr["floor_w"]) - kap * math.log(ref["f"])
               - math.log(energy_model.loop_energy(ref["ops"], pr) / ref["Q"]))
    for name, r in rows.items():
        f = energy_model.priced_clock({"ln_c": lnc_box, "kappa": kap}, pr, r["ops"], r["Q"], r["P"])
        assert abs(f / r["f"] - 1) < 0.02, (name, f, r["f"])


def test_committed_first_energy_model():
    """The first fit DESIGN §4 quotes (round 6's split variants on one box, priced with the
    synchronized probes of another, profiles/r06b_energy_model.json): kappa 2.39, round 3's split
    at -4.5% clock / +1.90% rate, and 70 splits ranked best (+0.27% over the build's 67)."""
    import json
    d = json.load(open(os.path.join(ROOT, "profiles", "r06b_energy_model.json")))
    rms, lnc, kap = energy_model.fit_priced(list(d["points"].values()), d["probe"])
    assert abs(kap - 2.39) < 0.01 and rms < 0.005
    r3 = d["priced"]["round3_split"]
    assert abs(r3["clock_change_pred"] + 0.045) < 0.002 and abs(r3["rate_change_pred"] - 0.019) < 0.002
    best, third = d["priced"]["split_ranking"]["best"], d["priced"]["split_ranking"]["every_third"]
    assert best["split"] == 70 and 0 < best["ghs"] / third["ghs"] - 1 < 0.005


def test_cpu_energy_counters(tmp_path, monkeypatch):
    """The CPU baseline's host energy: readable powercap counters are summed; a box without them
    (every MI355X box measured) gets None and the line says "not exposed"."""
    a, b = tmp_path / "package-0_energy_uj", tmp_path / "package-1_energy_uj"
    a.write_text("1000000\n")
    b.write_text("2500000\n")
    monkeypatch.setattr(bench.glob, "glob", lambda pat: [str(a), str(b)] if "powercap" in pat else [])
    assert bench.cpu_energy_counters() == {str(a): 1000000, str(b): 2500000}
    monkeypatch.setattr(bench.glob, "glob", lambda pat: [])
    assert bench.cpu_energy_counters() is None
