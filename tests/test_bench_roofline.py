"""CPU tests of bench.py's roofline line: `frac` is the
algorithm's per-nonce work over the VALU issue peak and cannot exceed 1;
SURVEY D4's pricing is reported beside it as `frac_survey_d4`; the dominant
kernel's registers come from the embedded code object.  Host only: the plan
(mh_plan) and the code-object metadata need no GPU."""
import pytest

import bench
import minehip
from minehip import codeobj

CUS = 256


def dominant_piece(cfg_name):
    cfg = bench.CONFIGS[cfg_name]
    lo, hi = bench.job_range(cfg, 1, 0, 1 if cfg["scaling"] == "weak" else 20)
    fast = [p for p in minehip.plan(cfg["msg"], lo, hi) if p["kind"] == 0]
    return max(fast, key=lambda p: p["count"] * p["nonce_slots"])


def kstat(p, ns):
    return {"name": f"mh::fast_search<{p['word']}, {p['mode']}>", "word": p["word"], "mode": p["mode"],
            "launches": 1, "nonces": p["count"], "ns": int(ns), "ops": p["count"] * p["nonce_ops"],
            "slots": p["count"] * p["nonce_slots"]}


def fastest_possible_ns(p, sclk=bench.PEAK_SCLK_HZ):
    """The shortest time the launch can take at the VALU issue limit: every SIMD quad-cycle
    issues two wave64 instructions, except that a half-rate one never shares its quad-cycle
    with another half-rate one -> >= max(H, N/2) quad-cycles per 64 nonces."""
    n, h = p["nonce_ops"], p["nonce_slots"] - p["nonce_ops"]
    quads = p["count"] / 64 * max(h, n / 2)
    return quads * 4 / (CUS * 4 * sclk) * 1e9


@pytest.mark.parametrize("cfg", ["2", "3a", "3b", "4"])
def test_frac_is_a_fraction_at_the_issue_limit(cfg):
    p = dominant_piece(cfg)
    line = bench.roofline([kstat(p, fastest_possible_ns(p))], CUS, 1)
    # at the fastest time the hardware allows, frac equals the mix bound, which is <= 1
    assert line["frac"] <= 1.0 and line["frac_physical"]
    assert line["frac"] == pytest.approx(line["mix_bound_frac"], rel=2e-3)
    assert line["frac_of_mix_bound"] == pytest.approx(1.0, rel=2e-3)
    assert line["alg_instr_per_nonce"] == p["nonce_ops"]
    # D4 prices a nonce at full compressions, so its ratio is larger (3b's exceeds 1)
    assert line["frac_survey_d4"] > line["frac"]
    if cfg == "3b":
        assert line["frac_survey_d4"] > 1.0


@pytest.mark.parametrize("cfg", ["2", "3a", "3b", "4"])
def test_frac_from_measured_kernel_rates(cfg):
    """The round-2 measured kernel rates (49.9 / 55.4 / 48.3 / 50.8 GH/s on
    the dominant kernel or better) give fractions in (0, 1)."""
    p = dominant_piece(cfg)
    for ghs in (30.0, 50.0, 60.0):
        line = bench.roofline([kstat(p, p["count"] / ghs)], CUS, 1)
        assert 0.0 < line["frac"] < 1.0, (cfg, ghs, line["frac"])
        assert line["frac"] == pytest.approx(ghs * 1e9 * p["nonce_ops"] / 1e12 / line["peak"], rel=1e-3)


def test_impossible_time_is_flagged():
    """A launch timed faster than the issue limit allows (work skipped, or a broken timer) gives
    frac > 1 and frac_physical False -- reported, not clipped."""
    p = dominant_piece("2")
    line = bench.roofline([kstat(p, fastest_possible_ns(p) * 0.5)], CUS, 1)
    assert line["frac"] > 1.0 and not line["frac_physical"]


def test_frac_recomputes_from_a_kernel_trace():
    """frac recomputed from a rocprofv3 kernel-trace average (profiles/
    r02at_kernel_stats.csv: fast_search<4,0> 70.08 ms over 3,294,967,000 nonces) is
    nonce_ops x nonces / avg / peak."""
    p = dominant_piece("2")
    assert (p["word"], p["mode"]) == (4, 0)
    line = bench.roofline([kstat(p, 70_080_409.8)], CUS, 1)
    want = p["nonce_ops"] * p["count"] / 0.0700804098 / 1e12 / (CUS * 128 * 2.4e9 / 1e12)
    assert line["frac"] == pytest.approx(want, rel=1e-3)
    assert line["frac"] < 0.75


def test_committed_summary_reproduces_frac():
    """the committed rocprof summary of a bench command
    (profiles/<tag>_kernel_stats_by_queue.csv, written by tools/trace_frac.py from that command's
    kernel trace: one row per (kernel, hardware queue), the coarse launches apart from the same
    kernel's tail-split launches) recomputes the committed line's roofline.frac within 1%."""
    import csv
    import glob
    import json
    import os
    import sys
    from conftest import ROOT
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import trace_frac
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_kernel_stats_by_queue.csv")))
    assert any("/r04" in f for f in found), "no round-4 summary committed"
    for f in found:
        tag = os.path.basename(f)[:-len("_kernel_stats_by_queue.csv")]
        line = json.load(open(os.path.join(ROOT, "profiles", f"{tag}_prof_bench.json")))
        stats = list(csv.DictReader(open(f)))
        frac, row = trace_frac.frac_from_stats(line, stats)
        assert line["roofline"]["kernel"].replace("mh::", "") in row["Name"]
        assert int(row["Lo_Digits"]) == line["roofline"]["lo_digits"]
        assert frac == pytest.approx(line["roofline"]["frac"], rel=0.01), (tag, frac)
        # and the per-kernel summary rocprofv3 writes cannot: it mixes both lane lengths
        names = [s for s in stats if s["Name"] == row["Name"]]
        assert len(names) >= 1


def test_resources_from_the_embedded_code_object():
    res = codeobj.fast_kernel_resources()
    from test_abi import KERNELS
    assert set(res) == KERNELS
    mix = bench.fast_loop_mix()
    for k, r in res.items():
        # the work-queue loop around the chunk body leaves a few bytes of spill in some layouts'
        # per-chunk setup (fast_search.hip min_waves; <8, OneEarly> at 7 waves: 48 B), never
        # inside the per-nonce loop
        assert r["scratch_bytes"] <= 48 and mix[k]["loop_spill_ops"] == 0, (k, r["scratch_bytes"])
        assert 32 <= r["vgpr"] <= 128 and r["agpr"] == 0, k
        assert r["max_waves_per_simd"] >= 4, k
    p = dominant_piece("2")
    line = bench.roofline([kstat(p, 7e7)], CUS, 1, res)
    assert line["resources"]["vgpr"] == res[(4, 0)]["vgpr"]
    assert codeobj.max_waves_per_simd(69) == 7 and codeobj.max_waves_per_simd(64) == 8
    assert codeobj.max_waves_per_simd(97) == 4 and codeobj.max_waves_per_simd(129) == 3


def test_msgpack_decoder_matches_the_msgpack_package():
    """codeobj's own MessagePack decoder (no dependency) against the msgpack package, on the
    embedded code object's metadata note and on a synthetic object with every type it handles."""
    msgpack = pytest.importorskip("msgpack")
    obj = {"a": [1, -1, 127, 128, -33, 65535, 2 ** 40, -(2 ** 40), 1.5, True, False, None],
           "s" * 40: "x" * 300, "b": b"\x00\x01", "m": {str(i): i for i in range(20)}, "l": list(range(40))}
    assert codeobj.unpack_msgpack(msgpack.packb(obj, use_bin_type=True)) == obj
    co = codeobj.fast_code_object()
    md = codeobj.metadata(co)
    assert md["amdhsa.target"].startswith("amdgcn-amd-amdhsa--gfx950")
    from test_abi import KERNELS
    assert len(md["amdhsa.kernels"]) == len(KERNELS)


def test_clock_probe_library_exports():
    """bench.py's in-kernel clock probe (tools/clock_probe.hip -> build/libclockprobe.so, part of
    `make all`): the two entry points bench.kernel_clock binds.  Loading needs no GPU."""
    import ctypes
    import os
    path = os.path.join(os.path.dirname(bench.__file__), "build", "libclockprobe.so")
    lib = ctypes.CDLL(path)
    assert hasattr(lib, "cp_start") and hasattr(lib, "cp_read")
    lib.cp_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    lib.cp_start.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int]
    buf = (ctypes.c_uint64 * 4)()
    assert lib.cp_read(0, buf, 1) == -1         # nothing started: refused, no device touched
    assert lib.cp_read(64, buf, 1) == -1        # no such device slot
    assert lib.cp_start(-1, 0.1, 0.1, 1) == -1  # refused before any HIP call


def test_kernel_clocks_one_thread_per_device():
    """The in-process N-GPU line reads every device's clock at once (bench.kernel_clocks): one host
    thread per distinct device, all probing concurrently, each with its own device's search; a
    failing probe leaves only that device's clock unknown.  Stub probe (no GPU)."""
    import threading
    import time
    seen, lock, inside = [], threading.Lock(), [0]
    peak = [0]

    def probe(search_dev, dev):
        with lock:
            inside[0] += 1
            peak[0] = max(peak[0], inside[0])
        time.sleep(0.05)
        search_dev(b"m", dev, dev)
        with lock:
            inside[0] -= 1
        if dev == 3:
            raise RuntimeError("no clock")
        return {"ghz": 2.0 + dev / 100}

    out = bench.kernel_clocks(lambda d: (lambda m, a, b: seen.append((d, a))), [0, 1, 1, 3, 0], probe=probe)
    assert sorted(out) == [0, 1, 3] and out[0]["ghz"] == 2.0 and out[1]["ghz"] == 2.01
    assert out[3]["ghz"] is None and "no clock" in out[3]["note"]
    assert sorted(seen) == [(0, 0), (1, 1), (3, 3)] and peak[0] == 3


@pytest.mark.gpu
def test_kernel_clock_during_a_search(gpu):
    """The probe's clock during an un-profiled fast_search<4, One> search: one reading per probe
    workgroup, spread over the 8 XCDs, inside MI355X's clock range."""
    kc = bench.kernel_clock(lambda m, a, b: gpu.search(m, a, b))
    assert kc is not None and kc["ghz"] is not None, kc
    assert 1.0 < kc["ghz"] <= 2.5, kc
    assert len(kc["ghz_by_xcd"]) == 8 and kc["probes"] == 64, kc
    assert all(1.0 < g <= 2.5 for g in kc["ghz_by_xcd"].values()), kc


def test_mix_bound_of_the_loop_as_built():
    """The build splits every third add3 (csrc/add3_split.py), so the per-nonce loop issues more
    instructions than nonce_ops and fewer half-rate ones; bench prices frac on nonce_ops and takes
    the reachable bound from the built loop (build/fast_loop_mix.json).  At the fastest time that
    loop allows, frac equals that bound, which is <= 1 and above the algorithm's own mix bound."""
    mix = bench.fast_loop_mix()
    from test_abi import KERNELS
    assert mix is not None and len(mix) == len(KERNELS)
    for cfg in ("2", "3a", "3b", "4"):
        p = dominant_piece(cfg)
        b = mix[(p["word"], p["mode"])]
        alg_half = p["nonce_slots"] - p["nonce_ops"]
        assert b["valu"] > p["nonce_ops"] and b["half"] < alg_half, (cfg, b)
        quads = p["count"] / 64 * max(b["half"], b["valu"] / 2)
        ns = quads * 4 / (CUS * 4 * bench.PEAK_SCLK_HZ) * 1e9
        line = bench.roofline([kstat(p, ns)], CUS, 1, None, mix)
        assert line["frac"] == pytest.approx(line["mix_bound_frac"], rel=2e-3)
        assert line["alg_mix_bound_frac"] < line["mix_bound_frac"] <= 1.0
        assert line["issued_loop"]["valu_per_nonce"] == b["valu"]


def test_fast_kernel_arguments_start_at_the_kernarg_segment():
    """fast_search's work-queue loop re-reads FastArgs through __builtin_amdgcn_kernarg_segment_ptr()
    (fast_search.hip), which assumes the by-value FastArgs is the first explicit argument at
    offset 0 and the partials pointer follows it.  Checked on every kernel of the embedded code
    object's metadata."""
    kernels = [k for k in codeobj.metadata(codeobj.fast_code_object())["amdhsa.kernels"]
               if k[".name"].startswith("_ZN2mh11fast_search")]
    from test_abi import KERNELS
    assert len(kernels) == len(KERNELS)
    for k in kernels:
        args = [a for a in k[".args"] if not a[".value_kind"].startswith("hidden_")]
        assert [a[".offset"] for a in args] == [0, args[0][".size"]], k[".name"]
        assert args[0][".value_kind"] == "by_value" and args[1][".value_kind"] == "global_buffer"
        assert args[0][".size"] % 8 == 0 and args[1][".size"] == 8


def test_clock_search_follows_the_dominant_layout():
    """The clock probe's search (and the line's energy window) runs the line's dominant kernel:
    configs[1]/[3]'s <4, One> keeps kernel_clock's default ("cmu440" from 10^11, 2^37 nonces);
    configs[2]'s messages get a bucket of their own layout, 2^36 nonces with a shorter window."""
    import inspect
    d = inspect.signature(bench.kernel_clock).parameters
    assert bench.clock_search("cmu440", 4, 0) == {"msg": "cmu440", "lo": d["lo"].default, "n": d["n"].default,
                                                  "delay_s": d["delay_s"].default, "window_s": d["window_s"].default}
    for msg, jm in (("a" * 100, (11, 0)), ("x" * 60, (0, 4))):
        cs = bench.clock_search(msg, *jm)
        assert cs and cs["n"] == 1 << 36 and cs["lo"] == 10 ** 10 and cs["delay_s"] + cs["window_s"] < 1.0
        import minehip
        got = {}
        for p in minehip.plan(msg, cs["lo"], cs["lo"] + cs["n"] - 1):
            if p["kind"] == 0:
                got[(p["word"], p["mode"])] = got.get((p["word"], p["mode"]), 0) + p["count"]
        assert max(got, key=got.get) == jm
    assert bench.clock_search("cmu440", 3, 0) is None  # d = 9's layout never fills 2^36 nonces
