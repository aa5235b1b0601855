"""tools/energy_probe.py -- price the fast kernel's instruction classes in joules at the power limit
 and record what the box exposes about energy and limits.

One process on one GPU (run on the box, after `make all`):

  python tools/energy_probe.py --tag r06a [--seconds 3] [--rounds 2] [--no-search]

  1. what amdsmi exposes (energy counter, limit accumulators, metrics; `amd-smi metric --help`);
  2. an idle window (no kernel);
  3. every probe of tools/valu_energy.hip (build/libvaluenergy.so): 8 waves per SIMD on every CU,
     all started together, running one instruction class for a fixed wall time, with the socket's
     energy counter and the limit accumulators read inside that time and a snapshot of power and
     per-XCD clocks in its middle;
  4. the product: a 2^37-nonce search of fast_search<4, One> with the in-kernel clock probe
     (bench.kernel_clock with an energy window), the figure bench.py reports as roofline.energy.

Per probe: wave-instructions per second (VALU and SALU, from every wave's own iteration count),
the clock the chip held (median over waves of shader cycles / 100 MHz ticks), joules, mean watts,
the share of the window each limit was active.  Rounds repeat the whole list, so drift shows.
Writes gpurun_out/<tag>/energy_probe.json; tools/energy_model.py fits the per-class prices.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd"), os.path.join(ROOT, "tools")]


def median(v):
    v = sorted(v)
    return v[len(v) // 2] if len(v) % 2 else (v[len(v) // 2 - 1] + v[len(v) // 2]) / 2


def run_probe(lib, meter, kind, seconds, nwg, dev=0, delay=1.0, margin=0.1):
    """One probe: every wave sleeps until `delay` after the launch, then runs its stream for
    `seconds`; the energy window is [start + margin, end - margin], inside the stream, with one
    metrics snapshot in its middle.  Rates come from every wave's own count over the stream."""
    import energy
    nw = 4 * nwg
    buf = (ctypes.c_uint64 * (4 * nw))()
    rc = lib.ve_start(dev, kind, delay, seconds, nwg)
    if rc != 0:
        return {"error": f"ve_start rc {rc}"}
    t0 = time.perf_counter()
    try:
        time.sleep(max(0.0, t0 + delay + margin - time.perf_counter()))
        a = meter.read()
        time.sleep(max(0.0, t0 + delay + seconds / 2 - time.perf_counter()))
        snap = meter.snapshot()
        time.sleep(max(0.0, t0 + delay + seconds - margin - time.perf_counter()))
        b = meter.read()
    finally:
        rc = lib.ve_wait(dev, buf, nwg)  # always: waits for the kernel and frees its buffer
    if rc != 0:
        return {"error": f"ve_wait rc {rc}"}
    res = energy.window_delta(a, b)
    res["snapshot"] = snap
    rows = [tuple(buf[4 * i:4 * i + 4]) for i in range(nw)]
    iters = sum(r[0] for r in rows)
    ghz = [r[1] / (r[2] / 1e8) / 1e9 for r in rows if r[2]]
    by_xcd = {}
    for r in rows:
        if r[2]:
            by_xcd.setdefault(int(r[3] & 0xffffffff), []).append(r[1] / (r[2] / 1e8) / 1e9)
    ticks = sorted(r[2] for r in rows)
    stream_s = median(ticks) / 1e8
    valu, salu = lib.ve_valu_per_iter(kind), lib.ve_salu_per_iter(kind)
    res.update({
        "kind": lib.ve_name(kind).decode(), "waves": nw, "stream_s": round(stream_s, 4),
        # every wave ran the same [start, end]: the shortest and longest stream show it
        "stream_s_range": [round(ticks[0] / 1e8, 4), round(ticks[-1] / 1e8, 4)],
        "clock_ghz": round(median(ghz), 4) if ghz else None,
        "clock_ghz_by_xcd": {str(x): round(median(v), 4) for x, v in sorted(by_xcd.items())},
        "wave_iterations": iters,
        "valu_wave_instr": iters * valu, "salu_wave_instr": iters * salu,
        "valu_wave_instr_per_s": iters * valu / stream_s if stream_s else None,
        "salu_wave_instr_per_s": iters * salu / stream_s if stream_s else None,
    })
    if res.get("valu_wave_instr_per_s") and res.get("clock_ghz"):
        # VALU instructions per SIMD quad-cycle (2 = the issue peak of a pair every quad)
        simds = 1024
        res["valu_per_simd_quad"] = round(res["valu_wave_instr_per_s"] / (simds * res["clock_ghz"] * 1e9 / 4), 4)
    return res


def idle_window(meter, seconds):
    import energy
    w = energy.Window(meter, snap_after_s=seconds / 2)
    with w:
        time.sleep(seconds)
    return dict(w.result, kind="idle")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r06_energy")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--nwg", type=int, default=0, help="workgroups (default: 8 per CU = 8 waves per SIMD)")
    ap.add_argument("--kinds", default="", help="comma-separated probe names (default: all)")
    ap.add_argument("--no-search", action="store_true")
    a = ap.parse_args()
    out_dir = os.path.join(ROOT, "gpurun_out", a.tag)
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, "energy_probe.json")

    import torch
    torch.cuda.set_device(0)
    import energy
    import bench
    import minehip
    meter = energy.meter_for_device(0)
    rep = {"tag": a.tag, "meter_ok": meter.ok, "meter_error": meter.error, "pci": list(meter.pci)}
    if meter.ok:
        rep["first_read"] = meter.read()
        rep["first_snapshot"] = meter.snapshot()
        for fn in ("amdsmi_get_power_cap_info", "amdsmi_get_power_info"):
            try:
                rep[fn] = {k: (v if isinstance(v, (int, float, str)) else str(v))
                           for k, v in getattr(meter.smi, fn)(meter.handle).items()}
            except Exception as e:
                rep[fn] = f"{type(e).__name__}: {e}"
    for args in (["metric", "--help"], ["static", "--limit"], ["metric", "--power", "--energy", "--throttle"]):
        try:
            r = subprocess.run(["amd-smi", *args], capture_output=True, text=True, timeout=30)
            rep["amd-smi " + " ".join(args)] = (r.stdout + r.stderr)[-6000:]
        except Exception as e:
            rep["amd-smi " + " ".join(args)] = f"{type(e).__name__}: {e}"
    json.dump(rep, open(path, "w"), indent=1)

    if not meter.ok:  # nothing to price without the energy counter: the report says why
        print(f"energy counter not available: {meter.error}; wrote {path}")
        return
    lib = ctypes.CDLL(os.path.join(ROOT, "build", "libvaluenergy.so"))
    lib.ve_name.restype = ctypes.c_char_p
    lib.ve_start.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int]
    lib.ve_wait.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    nwg = a.nwg or 8 * cus
    kinds = [k for k in range(lib.ve_kinds())
             if not a.kinds or lib.ve_name(k).decode() in a.kinds.split(",")]
    minehip.search("cmu440", 10 ** 9, 10 ** 9 + (1 << 30))  # module load, clocks up
    rep["rounds"] = []
    for rnd in range(a.rounds):
        rows = [idle_window(meter, 2.0)]
        for k in kinds:
            r = run_probe(lib, meter, k, a.seconds, nwg)
            rows.append(r)
            print(json.dumps({x: r.get(x) for x in ("kind", "clock_ghz", "mean_w", "limiter", "valu_per_simd_quad")}),
                  flush=True)
            time.sleep(0.5)
        if not a.no_search:
            kc = bench.kernel_clock(lambda m, lo, hi: minehip.search(m, lo, hi), 0, meter=meter)
            rows.append({"kind": "product_fast_search<4,One>", "kernel_clock": kc})
            print(json.dumps({"kind": "product", "ghz": (kc or {}).get("ghz"),
                              "energy": (kc or {}).get("energy")}), flush=True)
        rep["rounds"].append(rows)
        json.dump(rep, open(path, "w"), indent=1)
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
