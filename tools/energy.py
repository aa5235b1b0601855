"""tools/energy.py -- the energy a search costs, the power it draws and the limit that holds the
clock, read from the GPU's power-management firmware through amdsmi (the Python binding of
amd-smi that ships in /opt/rocm; measurement only, never part of the product library).

Why: the fast kernel runs at the package power limit, so the clock -- and with it GH/s -- is set
by the energy each nonce costs.  Three readings, each before
and after a window of work:

  * the socket's accumulated energy counter (`amdsmi_get_energy_count`: ticks x resolution uJ),
    so energy and mean power over the window need no sampling;
  * the firmware's violation accumulators (`amdsmi_get_violation_status`: `acc_ppt_pwr` = package
    power limit, `acc_socket_thrm`, `acc_vr_thrm`, `acc_hbm_thrm`, `acc_prochot_thrm`, and
    `acc_gfx_clk_below_host_limit`, against the tick counter `acc_counter`): the share of the
    window each limit was active, so a line names which one held the clock;
  * a mid-window snapshot of `amdsmi_get_gpu_metrics_info` (GFX voltage, current socket power,
    per-XCD GFX clocks, throttle status bits).

Every field the device or the library does not expose is reported as missing, never guessed.
The GPU is matched by PCI address (the HIP device's domain:bus:device), not by index.
"""
import threading
import time

_LOCK = threading.Lock()   # amdsmi calls from the in-process path's per-device threads
_STATE = {"init": False, "error": None}

LIMITS = ("ppt_pwr", "socket_thrm", "vr_thrm", "hbm_thrm", "prochot_thrm", "gfx_clk_below_host_limit")


def _amdsmi():
    with _LOCK:
        if _STATE["init"]:
            return _STATE["mod"]
        if _STATE["error"]:
            return None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            _STATE["mod"] = amdsmi
            _STATE["init"] = True
            return amdsmi
        except Exception as e:  # no library, no driver, no permission: energy not exposed
            _STATE["error"] = f"amdsmi unavailable: {type(e).__name__}: {e}"
            return None


def unavailable_reason():
    return _STATE["error"]


def _int(v):
    return v if isinstance(v, int) and not isinstance(v, bool) else None


def parse_bdf(s):
    """'0000:75:00.0' -> (domain, bus, device)."""
    dom, bus, rest = s.strip().split(":")
    return int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)


class Meter:
    """One GPU's energy counter, limit accumulators and metrics.  pci = (domain, bus, device) of
    the HIP device (torch.cuda.get_device_properties: pci_domain_id, pci_bus_id, pci_device_id)."""

    def __init__(self, pci):
        self.pci = tuple(pci)
        self.handle = None
        self.error = None
        smi = _amdsmi()
        if smi is None:
            self.error = unavailable_reason()
            return
        self.smi = smi
        try:
            with _LOCK:
                for h in smi.amdsmi_get_processor_handles():
                    if parse_bdf(smi.amdsmi_get_gpu_device_bdf(h)) == self.pci:
                        self.handle = h
                        break
        except Exception as e:
            self.error = f"amdsmi handles: {type(e).__name__}: {e}"
            return
        if self.handle is None:
            self.error = f"no amdsmi GPU at PCI {self.pci}"

    @property
    def ok(self):
        return self.handle is not None

    def _call(self, fn):
        try:
            with _LOCK:
                return fn(self.handle), None
        except Exception as e:
            return None, f"{type(e).__name__}: {e}"

    def read(self):
        """Counters at one instant: host time, energy (J), limit accumulators."""
        out = {"host_ns": time.perf_counter_ns()}
        e, err = self._call(self.smi.amdsmi_get_energy_count)
        if e and _int(e.get("energy_accumulator")) is not None:
            res = float(e.get("counter_resolution") or 0.0)
            out["energy_j"] = e["energy_accumulator"] * res * 1e-6
            out["energy_ts"] = _int(e.get("timestamp"))
            out["energy_res_uj"] = res
        else:
            out["energy_error"] = err or "energy counter not exposed"
        v, err = self._call(self.smi.amdsmi_get_violation_status)
        if v:
            out["viol"] = {k: _int(v.get(k)) for k in ("acc_counter",) + tuple("acc_" + x for x in LIMITS)}
        else:
            out["viol_error"] = err
        return out

    def snapshot(self):
        """Instantaneous metrics (voltage, power, per-XCD clocks, throttle bits, limit)."""
        out = {}
        m, err = self._call(self.smi.amdsmi_get_gpu_metrics_info)
        if m:
            for k in ("voltage_gfx", "voltage_soc", "voltage_mem", "current_socket_power", "average_socket_power",
                      "temperature_hotspot", "temperature_mem", "throttle_status", "indep_throttle_status",
                      "average_gfxclk_frequency"):
                val = m.get(k)
                if isinstance(val, (int, float)) and not isinstance(val, bool):
                    out[k] = val
            clks = [c for c in (m.get("current_gfxclks") or []) if _int(c) and c < 0xFFFF]
            if clks:
                out["gfx_clk_mhz"] = clks
        else:
            out["metrics_error"] = err
        p, err = self._call(self.smi.amdsmi_get_power_info)
        if p:
            lim = p.get("power_limit")
            if _int(lim):
                # amdsmi reports the limit in W on gfx950 (uW on older parts)
                out["power_limit_w"] = lim / 1e6 if lim > 100000 else lim
        return out


def window_delta(a, b, nonces=None):
    """Energy, mean power and the share of the window each limit was active, between two reads."""
    sec = (b["host_ns"] - a["host_ns"]) * 1e-9
    out = {"seconds": round(sec, 4)}
    if "energy_j" in a and "energy_j" in b:
        j = b["energy_j"] - a["energy_j"]
        if a.get("energy_ts") and b.get("energy_ts") and b["energy_ts"] > a["energy_ts"]:
            # the firmware's own timestamps of the two readings (ns), when it gives them
            fw = (b["energy_ts"] - a["energy_ts"]) * 1e-9
            if 0.5 * sec < fw < 2 * sec:
                out["fw_seconds"] = round(fw, 4)
        out["joules"] = round(j, 3)
        out["mean_w"] = round(j / sec, 1) if sec > 0 else None
        if nonces:
            out["nonces"] = nonces
            out["j_per_gnonce"] = round(j / (nonces / 1e9), 4)
    else:
        out["energy_error"] = a.get("energy_error") or b.get("energy_error") or "energy counter not exposed"
    va, vb = a.get("viol"), b.get("viol")
    if va and vb and va.get("acc_counter") is not None and vb.get("acc_counter") is not None:
        ticks = vb["acc_counter"] - va["acc_counter"]
        res = {}
        for x in LIMITS:
            k = "acc_" + x
            if va.get(k) is not None and vb.get(k) is not None and ticks > 0:
                res[x] = round((vb[k] - va[k]) / ticks, 4)
        out["limit_active_share"] = res
        out["limit_ticks"] = ticks
        top = max(res.items(), key=lambda kv: kv[1]) if res else None
        out["limiter"] = (top[0] if top and top[1] >= 0.05 else
                          "none reported" if res else "not exposed")
    else:
        out["limiter"] = "not exposed"
        out["limit_error"] = a.get("viol_error") or b.get("viol_error") or "violation accumulators not exposed"
    return out


class Window:
    """with Window(meter, nonces) as w: <work>  -> w.result: window_delta plus one metrics
    snapshot taken mid-window (after `snap_after_s`)."""

    def __init__(self, meter, nonces=None, snap_after_s=0.6):
        self.meter, self.nonces, self.snap_after_s = meter, nonces, snap_after_s
        self.result = None
        self._snap = {}
        self._timer = None

    def __enter__(self):
        if self.meter is not None and self.meter.ok:
            self.a = self.meter.read()
            self._timer = threading.Timer(self.snap_after_s, lambda: self._snap.update(self.meter.snapshot()))
            self._timer.start()
        return self

    def __exit__(self, *exc):
        if self.meter is None or not self.meter.ok:
            self.result = {"error": getattr(self.meter, "error", None) or "no meter"}
            return False
        b = self.meter.read()
        self._timer.cancel()
        self._timer.join()
        self.result = window_delta(self.a, b, self.nonces)
        if self._snap:
            self.result["snapshot"] = dict(self._snap)
        return False


def _loaded_hip():
    """The HIP runtime this process already uses (its path from /proc/self/maps), or None: asking
    a second copy of the runtime would initialise another HIP instance in the process."""
    import ctypes
    try:
        for line in open("/proc/self/maps"):
            path = line.split()[-1] if len(line.split()) >= 6 else ""
            if "libamdhip64.so" in path:
                return ctypes.CDLL(path)
    except OSError:
        pass
    return None


def pci_of_device(dev):
    """(domain, bus, device) of HIP device `dev`: hipDeviceGetPCIBusId from the runtime already
    loaded (libminehip's or torch's), else torch's device properties."""
    import ctypes
    hip = _loaded_hip()
    if hip is not None:
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, ctypes.c_int(dev)) == 0:
            return parse_bdf(buf.value.decode())
    import torch
    p = torch.cuda.get_device_properties(dev)
    return p.pci_domain_id, p.pci_bus_id, p.pci_device_id


def meter_for_device(dev):
    """A Meter for HIP device `dev`, found by its PCI address."""
    return Meter(pci_of_device(dev))
