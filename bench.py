#!/usr/bin/env python3
"""bench.py -- SHA-256 nonce-search throughput (BASELINE.json metric: GH/s at
1/2/4/8 MI355X and % of the VALU integer roofline).

A step is one search -- the miner's scan over bitcoin.Hash (reference
bitcoin/hash.go:13-17; loop spec SURVEY.md §8(a) A2, stub bitcoin/miner/miner.go:33)
-- of one batch of nonces, ending in the 16-byte (hash, nonce) host merge.

Workloads (BASELINE.json configs; `--config` overrides the default):
  N = 1  "2"  configs[1]: msg "cmu440", nonces [0, 2^32-1] every step (all
              decimal buckets d = 1..10).  The metric's single-GPU line.
  N > 1  "4"  configs[3]: msg "cmu440", nonces [0, 2^40-1] sharded over the N
              GPUs with a host min-merge -- strong scaling.  The K timed steps
              cover [0, 2^40-1] exactly once: step k scans the k-th of K equal
              slices, split into N contiguous shards.  The merged result of the
              timed region is configs[3]'s answer.
  "3a"/"3b"   configs[2] (100 x 'a': host midstate; 60 x 'x': two tail blocks).

How the N GPUs are driven (no RCCL, one 16-byte tuple per
shard, merged on the host):
  * launched (WORLD_SIZE > 1, e.g. `torch.distributed.run --nproc-per-node N
    bench.py --gpus N`): one process per GPU -- the "one miner process per GPU"
    layout of configs[4].  Rank r searches its shard on device LOCAL_RANK with
    mh_search; the tuples, the barrier and the max-over-ranks time go over a
    gloo (host) process group.  Each step's merge is posted asynchronously and
    completes while the next step searches (LaunchedSteps); all of them complete
    inside the timed region.  WORLD_SIZE must equal --gpus.
  * self-contained (`python bench.py --gpus N`, no launcher): one process, one
    host thread + HIP stream per device, mh_search_multi over devices 0..N-1:
    each step is one contiguous shard per device, sized by the device's rate
    measured on the earlier steps (the library keeps the rates), merged on the
    host.  Fewer than N visible devices is an error: exit 2, no JSON line.
    `--multi` forces this path at N = 1.
Every line carries `n1_config4_ghs`, one configs[3] step searched on one device
alone, and configs[3] lines `per_gpu_efficiency` = value / (N x it).

Rank 0 prints ONE JSON line.  `roofline.frac` is the dominant kernel's
algorithmic per-nonce work (nonce_ops: the VALU instructions one nonce needs
after hoisting, SURVEY §8(d) D4 restated for gfx950) x nonces over its
HIP-event launch time, against the VALU issue peak: 2 instructions per SIMD
quad-cycle = 256 CU x 128 lanes/clk x 2.4 GHz.  It cannot
exceed 1.  `roofline.frac_survey_d4` prices a nonce at SURVEY D4's 1,616 ops
per compression instead (can exceed 1).  `roofline.resources` are the kernel's
VGPR/SGPR/scratch from the embedded code object.  At N = 1, rocprofv3 --pmc
passes over one launch of each of the two largest kernels give HBM traffic,
the clock (`sclk_ghz`, `roofline.frac_at_sclk`) and the SQ counters
(`roofline.pmc`); probe workgroups on their own stream read the clock inside the GPU
during an un-profiled search (`roofline.kernel_clock`, `frac_at_kernel_clk`,
tools/clock_probe.hip).  `cpu_baseline` times the CPU port of the reference loop
(oracle/) on a bounded sample, at N = 1 only.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "bitcoin-miner_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "GH/s (SHA-256 nonce search) at 1/2/4/8 MI355X; % of VALU int roofline"
PEAK_SCLK_HZ = 2.4e9          # MI355X max engine clock (MI355X_MICROARCH.md chip table)
# VALU peak: 4 SIMD-32 per CU, a wave64 instruction every 2 cycles = 128
# int32 lane-ops/clk/CU (MI355X_MICROARCH.md "Wave scheduling").
LANES_PER_CU_CLK = 128
# canonical gfx950 VALU ops of one SHA-256 compression.
# Ops per hash = 1,616 x tail blocks; host-midstate blocks are excluded.
SURVEY_OPS_PER_COMPRESSION = 1616
OPS_PER_BLOCK = 1376          # this kernel's count for an un-hoisted compression (v_bitop3 xor3)

# BASELINE.json configs as bench workloads.
CONFIGS = {
    "2": dict(msg="cmu440", bits=32, scaling="weak",
              desc="BASELINE configs[1]: single SHA block, nonces [0, 2^32-1] per GPU per step "
                   "(all buckets d=1..10 at N=1)"),
    "3a": dict(msg="a" * 100, bits=34, scaling="weak",
               desc="BASELINE configs[2]: 100-byte msg (host midstate block), 2^34 nonces per GPU per step"),
    "3b": dict(msg="x" * 60, bits=34, scaling="weak",
               desc="BASELINE configs[2]: 60-byte msg (two tail blocks), 2^34 nonces per GPU per step"),
    "4": dict(msg="cmu440", bits=40, scaling="strong",
              desc="BASELINE configs[3]: nonces [0, 2^40-1] sharded over the GPUs, host min-merge; "
                   "the K timed steps are K equal slices covering the range once"),
}


def default_config(gpus):
    return "2" if gpus == 1 else "4"


def shard(rank, bits):
    lo = rank << bits
    return lo, lo + (1 << bits) - 1


def split(lo, hi, parts, i):
    """The i-th of `parts` contiguous, near-equal pieces of [lo, hi] (None if empty)."""
    n = hi - lo + 1
    a = lo + n * i // parts
    b = lo + n * (i + 1) // parts - 1
    return (a, b) if b >= a else None


def step_range(cfg, k, steps):
    """The whole nonce range of step k (all ranks together).  Weak configs scan
    the same [0, N*2^bits) every step (the caller splits it per GPU); the strong
    config's K steps are K slices of [0, 2^bits)."""
    if cfg["scaling"] == "weak":
        return None
    return split(0, (1 << cfg["bits"]) - 1, steps, k % steps)


def weighted_split(lo, hi, weights, i):
    """The i-th of len(weights) contiguous pieces of [lo, hi], piece j sized in proportion to
    the integer weights[j] (None if empty).  Exact integer arithmetic: the pieces tile [lo, hi]."""
    n = hi - lo + 1
    tot = sum(weights)
    before = sum(weights[:i])
    a = lo + n * before // tot
    b = lo + n * (before + weights[i]) // tot - 1
    return (a, b) if b >= a else None


def rank_range(cfg, rank, world, k=0, steps=1, weights=None):
    """This rank's shard of step k.  Strong steps are split equally, or in proportion to
    `weights` (one integer per rank, Balancer.weights) when given."""
    if cfg["scaling"] == "weak":
        return shard(rank, cfg["bits"])
    if weights is not None:
        return weighted_split(*step_range(cfg, k, steps), weights, rank)
    return split(*step_range(cfg, k, steps), world, rank)


def job_range(cfg, world, k=0, steps=1):
    """Every rank's shard of step k together."""
    if cfg["scaling"] == "weak":
        return 0, (world << cfg["bits"]) - 1
    return step_range(cfg, k, steps)


def merge(results):
    """Lexicographic (hash, nonce) minimum == the reference loop's strict-< first min."""
    return min(results)


class Balancer:
    """Strong-scaling shard sizes in proportion to each rank's measured search rate.

    Equal shards make every strong step as slow as the slowest GPU, and MI355X
    devices run this power-limited kernel at clocks that differ by several
    percent.  Each rank's (nonces, search ns) of a step ride
    in that step's merge all_gather, so every rank holds the same cumulative
    rates and computes the same split: no extra collective, and the K steps
    still tile the job range exactly once.  The first step a rank sees (device
    context and module load) is not counted."""

    SCALE = 1 << 20

    def __init__(self, world, enabled=True):
        self.world = world
        self.enabled = enabled and world > 1
        self.nonces = [0] * world
        self.ns = [0] * world
        self.steps_seen = 0

    def update(self, stats):
        self.steps_seen += 1
        if self.steps_seen == 1:
            return
        for i, (n, t) in enumerate(stats):
            self.nonces[i] += n
            self.ns[i] += t

    def weights(self):
        """Integer weights (one per rank, max SCALE), or None for equal shards."""
        if not self.enabled or any(n <= 0 or t <= 0 for n, t in zip(self.nonces, self.ns)):
            return None
        rates = [n / t for n, t in zip(self.nonces, self.ns)]
        top = max(rates)
        return [max(1, round(self.SCALE * x / top)) for x in rates]


class LaunchedSteps:
    """The steps of the launched (one process per GPU) path, pipelined.  Step k searches this
    rank's shard of step k (rate-weighted when `bal` has rates) with search(lo, hi) and posts the
    step's host merge -- the 16-byte tuple and (nonces, search ns) of every rank, one gloo
    all_gather -- without waiting for it: the merge of step k runs on gloo's thread while step
    k + 1 searches.  So a rank that finishes a step early starts the next one instead of waiting
    for the slowest rank, and the merge's latency leaves the critical path; every merge is
    complete before the timed region ends (finish()).  Step k's shards are sized from the merges
    of steps <= k - 2, which every rank has folded before cutting step k, so all ranks cut the
    same shards and the K steps still tile the job exactly once."""

    def __init__(self, search, cfg, rank, world, steps, dist, bal=None):
        self.search, self.cfg, self.rank, self.world, self.steps = search, cfg, rank, world, steps
        self.dist, self.bal = dist, bal
        self.pending = []  # [(k, work, gathered tensors)] in step order
        self.best = None
        self.nonces = 0    # this rank's nonces since the last finish()

    def _fold(self, item):
        k, work, out = item[:3]
        if work is not None:
            work.wait()
            vals = [o.tolist() for o in out]
        else:
            vals = [out]
        merged = merge((v[0] + (1 << 63), v[1] + (1 << 63)) for v in vals)
        self.best = merged if self.best is None else merge([self.best, merged])
        if self.bal is not None:
            self.bal.update([(v[2], v[3]) for v in vals])

    def step(self, k):
        while self.pending and self.pending[0][0] <= k - 2:
            self._fold(self.pending.pop(0))
        rr = rank_range(self.cfg, self.rank, self.world, k, self.steps,
                        self.bal.weights() if self.bal is not None else None)
        t0 = time.perf_counter_ns()
        r = self.search(rr[0], rr[1]) if rr else ((1 << 64) - 1, (1 << 64) - 1)
        dt = time.perf_counter_ns() - t0
        n = rr[1] - rr[0] + 1 if rr else 0
        self.nonces += n
        v = [r[0] - (1 << 63), r[1] - (1 << 63), n, dt]  # u64 -> i64, order kept
        if self.world == 1:
            self.pending.append((k, None, v))
            return
        import torch
        t = torch.tensor(v, dtype=torch.int64)
        out = [torch.empty_like(t) for _ in range(self.world)]
        # the input tensor rides along with the outputs: both stay alive until the merge is folded
        self.pending.append((k, self.dist.all_gather(out, t, async_op=True), out, t))

    def finish(self):
        """Complete every posted merge; returns the merged (hash, nonce) of the steps since the
        last finish() and resets it (and the nonce count) for the next region."""
        while self.pending:
            self._fold(self.pending.pop(0))
        best, self.best = self.best, None
        return best


def run_timed(step, steps, warmup, barrier, sync, finish=None):
    """W untimed warmup steps, then exactly `steps` timed steps between a barrier
    + device sync on both sides.  step(k) returns the merged (hash, nonce) of
    step k, or None when its merge is still in flight: then finish() completes
    the outstanding merges and returns their minimum (inside the timed region).
    Returns (min over the timed steps, this rank's elapsed seconds)."""
    for w in range(warmup):
        step(w)
    if finish is not None:
        finish()  # the warmup's merges: complete, and not part of the timed result
    barrier()
    sync()
    t0 = time.perf_counter()
    best = None
    for k in range(steps):
        r = step(k)
        if r is not None:
            best = r if best is None else merge([best, r])
    if finish is not None:
        r = finish()
        if r is not None:
            best = r if best is None else merge([best, r])
    barrier()
    sync()
    return best, time.perf_counter() - t0


def golden_expect(msg, lo, hi):
    """The expected (hash, nonce) of [lo, hi] from the full-size fixtures
    (tests/golden/fullsize_*.json, scanned on the CPU by gen_fullsize.py /
    gen_cfg4.py) when [lo, hi] is a union of their chunks; None otherwise.
    Data only: no oracle code runs here."""
    for path in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "fullsize_*.json"))):
        with open(path) as f:
            d = json.load(f)
        if bytes.fromhex(d["msg_hex"]) != msg:
            continue
        for s_lo, s_hi, h, n in d.get("samples", []):  # sampled chunks (fullsize_cfg4s.json)
            if (s_lo, s_hi) == (lo, hi):
                return (h, n)
        if "chunks" not in d:
            continue
        size = 1 << d["chunk_bits"]
        if lo < d["lo"] or hi > d["hi"]:
            continue
        if (lo - d["lo"]) % size or (hi + 1 - d["lo"]) % size:
            continue
        i, j = (lo - d["lo"]) // size, (hi + 1 - d["lo"]) // size
        return min(tuple(c) for c in d["chunks"][i:j])
    return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_cpu_quota():
    """CPUs the cgroup quota allows this process (cgroup v2 cpu.max, v1 cfs files), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, q // p)
    except (OSError, ValueError):
        return None


def cpu_threads():
    """Threads for the CPU baseline and how they were chosen.  Every core this process may run on
    (its affinity mask), capped by a cgroup CPU quota and by the job's CPU share: the GPU box
    exports OMP_NUM_THREADS as each one-GPU job's share of a much larger machine (its affinity
    shows every core of the node), and a job must not run more threads than that.
    BENCH_CPU_THREADS overrides.  Returns (threads, facts for the line)."""
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpu_quota()
    omp = os.environ.get("OMP_NUM_THREADS")
    share = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    facts = {"cores_available": avail, "cgroup_quota_cores": quota, "job_cpu_share": share}
    if os.environ.get("BENCH_CPU_THREADS"):
        facts["cores_rule"] = "BENCH_CPU_THREADS"
        return max(1, int(os.environ["BENCH_CPU_THREADS"])), facts
    t = min(x for x in (avail, quota, share) if x)
    facts["cores_rule"] = ("min(affinity cores, cgroup quota, the job's CPU share OMP_NUM_THREADS)"
                           if t < avail else "every core in the affinity mask")
    return t, facts


def cpu_energy_counters():
    """Readable host-CPU package energy counters (powercap / RAPL: {path: microjoules}), or None.
    The MI355X boxes measured so far expose none (no powercap class; k10temp has temperatures
    only), and the line then says so."""
    paths = sorted(glob.glob("/sys/class/powercap/*/energy_uj"))
    out = {}
    for p in paths:
        try:
            out[p] = int(open(p).read())
        except (OSError, ValueError):
            return None
    return out or None


def cpu_baseline(msg, threads):
    """The reference loop ported to C (oracle/): per nonce format "%s %d" and a
    full SHA-256 from the IV, like bitcoin/hash.go.  Bounded sample of the
    same workload (d = 10 nonces, the bulk of configs[1])."""
    from oracle import oracle
    base = 10 ** 9
    n1 = 6_000_000
    t = time.perf_counter()
    oracle.search(msg, base, base + n1 - 1, threads=1)
    st = n1 / (time.perf_counter() - t)
    nT = 12_000_000 * threads
    e0 = cpu_energy_counters()
    t = time.perf_counter()
    oracle.search(msg, base, base + nT - 1, threads=threads)
    mt = nT / (time.perf_counter() - t)
    e1 = cpu_energy_counters() if e0 else None
    if e0 and e1 and set(e0) == set(e1):
        # package counters wrap; a window this short wraps at most once, and then it shows as negative
        joules = sum(e1[k] - e0[k] for k in e0) * 1e-6
        energy = ({"j_per_gnonce": round(joules / (nT / 1e9), 2), "joules": round(joules, 2),
                   "counters": len(e0), "note": "host package energy (powercap), the whole socket(s)"}
                  if joules > 0 else {"error": "a counter wrapped inside the window"})
    else:
        energy = "not exposed (no readable powercap / RAPL energy counter on this host)"
    # BASELINE configs[0] ("cmu440", nonces 0..9,999,999) timed in full
    t = time.perf_counter()
    c1 = oracle.search("cmu440", 0, 9_999_999, threads=threads)
    c1_ms = (time.perf_counter() - t) * 1e3
    # a tuned CPU miner on the same cores: midstate + OpenSSL SHA-256 (SHA-NI), oracle/openssl_scan.c
    nO = 50_000_000 * threads
    t = time.perf_counter()
    oracle.search_openssl(msg, base, base + nO - 1, threads=threads)
    opt = nO / (time.perf_counter() - t)
    return {
        "value": mt / 1e9, "unit": "GH/s", "cores": threads, "kind": "port",
        "sample": f"msg {msg!r}, nonces [1e9, 1e9+{nT}) on {threads} threads "
                  f"({cpu_model()}); single thread {n1} nonces: {st / 1e6:.3f} MH/s",
        "single_thread_value": st / 1e9,
        # J per 10^9 nonces of the multi-threaded run, beside the GPU's roofline.energy
        "energy": energy,
        "config1_ms": round(c1_ms, 1), "config1_result": list(c1),
        "optimized": {"value": opt / 1e9, "unit": "GH/s", "cores": threads,
                      "kind": "midstate + OpenSSL SHA-256 (oracle/openssl_scan.c), not the reference's loop",
                      "sample": f"nonces [1e9, 1e9+{nO})"},
    }


def largest_piece(msg, lo, hi, var):
    """The largest launch of fast_search<word, mode> with var's lane length in the plan of [lo, hi]."""
    import minehip
    ps = [p for p in minehip.plan(msg, lo, hi)
          if p["kind"] == 0 and p["word"] == var["word"] and p["mode"] == var["mode"]
          and p["lo_digits"] == var.get("lo_digits", p["lo_digits"])]
    return max(ps, key=lambda p: p["count"]) if ps else None


# rocprofv3 --pmc passes: one block-limited counter set per run
# (MI355X_MICROARCH.md: 8 SQ, 4 TCC -- FETCH_SIZE takes 3, WRITE_SIZE 2 --, 2 GRBM).
PMC_PASSES = (
    ("FETCH_SIZE",),
    ("WRITE_SIZE",),
    ("GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"),
    ("GRBM_GUI_ACTIVE", "SQ_ACTIVE_INST_ANY", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_SALU",
     "SQ_ACTIVE_INST_SCA", "SQ_INSTS_VALU_INT32", "SQ_IFETCH", "SQ_BUSY_CU_CYCLES", "SQ_CYCLES"),
)


def pmc_counters(msg, pieces, dev, timeout=90, passes=PMC_PASSES):
    """PMC counters of ONE launch of each given piece: one rocprofv3 --pmc run
    per counter set over a child process (tools/pmc_launch.py) that searches
    exactly those launches' nonces.  Returns ({kernel name: {counter: value,
    "dur_ns": ..., "cycles": ...}}, error)."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    names = [f"fast_search<{p['word']}, {p['mode']}>" for p in pieces]
    ranges = [f"{p['first']}:{p['first'] + p['count'] - 1}:{p['lo_digits']}" for p in pieces]
    vals = {n: {} for n in names}
    work = tempfile.mkdtemp(prefix="bench_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        for counters in passes:
            out = os.path.join(work, f"p{passes.index(counters)}")
            cmd = [prof, "--pmc", *counters, "-d", out, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.join(ROOT, "tools", "pmc_launch.py"), msg, str(dev), *ranges]
            try:
                rc = subprocess.run(cmd, cwd="/tmp", env=env, timeout=timeout, stdout=subprocess.DEVNULL,
                                    stderr=subprocess.PIPE).returncode
            except subprocess.TimeoutExpired:
                return None, f"rocprofv3 --pmc {' '.join(counters)} timed out"
            files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
            if rc != 0 or not files:
                return None, f"rocprofv3 --pmc {' '.join(counters)} failed (rc {rc})"
            per = {}
            for r in csv.DictReader(open(files[0])):
                name = next((n for n in names if n in r["Kernel_Name"]), None)
                if name is None or r["Counter_Name"] not in counters:
                    continue
                d = per.setdefault((name, r["Dispatch_Id"]), {})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                d["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for n in names:
                ds = [v for (k, _), v in per.items() if k == n]
                if len(ds) != 1:
                    return None, f"{len(ds)} {n} dispatches in the --pmc {' '.join(counters)} pass, expected 1"
                if "GRBM_GUI_ACTIVE" in ds[0]:  # per-pass clock, kept per pass
                    ds[0][f"GRBM_GUI_ACTIVE@{passes.index(counters)}"] = ds[0].pop("GRBM_GUI_ACTIVE")
                    ds[0][f"dur_ns@{passes.index(counters)}"] = ds[0]["dur_ns"]
                vals[n].update(ds[0])
    finally:
        shutil.rmtree(work, ignore_errors=True)
    return vals, None


def pmc_derived(v, piece, cus):
    """Per-launch PMC figures of one fast_search launch (raw counters kept).
    SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_* count quad-cycles summed over
    waves; GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md)."""
    g, dur = v["GRBM_GUI_ACTIVE@2"], v["dur_ns@2"]
    cycles = g / 8                       # shader clocks the launch took
    simds = cus * 4
    nonces = piece["count"]
    wc = v["SQ_WAVE_CYCLES"]
    out = {
        "sclk_ghz": round(cycles / dur, 3),
        "pmc_launch_ms": round(dur / 1e6, 3),
        "nonces": nonces,
        "valu_instr_per_nonce": round(v["SQ_INSTS_VALU"] * 64 / nonces, 1),
        # SIMD cycles per issued wave64 VALU instruction (2 = two per quad-cycle, the issue peak)
        "cycles_per_valu_instr": round(cycles * simds / v["SQ_INSTS_VALU"], 3),
        # mean resident waves per SIMD over the launch (occupancy)
        "waves_per_simd": round(wc * 4 / (cycles * simds), 2),
        "waves": int(v["SQ_WAVES"]),
        # share of wave lifetime: issuing VALU / stalled on issue / parked on a wait
        "valu_active_of_wave_cycles": round(v["SQ_ACTIVE_INST_VALU"] / wc, 4),
        "wait_inst_any_of_wave_cycles": round(v["SQ_WAIT_INST_ANY"] / wc, 4),
        "wait_any_of_wave_cycles": round(v["SQ_WAIT_ANY"] / wc, 4),
        # VALU instructions issued per SIMD quad-cycle (SQ_ACTIVE_INST_VALU counts one per instruction,
        # calibrated on tools/gen_valu_pair.py probes): 1 = one per quad, 2 = a pair in every quad
        "valu_instr_per_quad": round(v["SQ_ACTIVE_INST_VALU"] * 4 / (cycles * simds), 4),
        # quad-cycles in which a SIMD issued two VALU instructions, per SIMD quad-cycle
        "valu2_of_simd_quads": round(v["SQ_ACTIVE_INST_VALU2"] / (cycles * simds / 4), 4),
        "counters": {k: v[k] for k in sorted(v) if not k.startswith("dur_ns")},
    }
    if "GRBM_GUI_ACTIVE@3" in v:
        out["sclk_ghz_pass4"] = round(v["GRBM_GUI_ACTIVE@3"] / 8 / v["dur_ns@3"], 3)
        out["salu_instr_per_nonce"] = round(v["SQ_INSTS_SALU"] * 64 / nonces, 2)
    return out


def gpu_config1(search_dev):
    """BASELINE configs[0] on the GPU: wall ms of one [0, 9,999,999] search (median of 10)."""
    search_dev("cmu440", 0, 9_999_999)
    ts = []
    for _ in range(10):
        t = time.perf_counter()
        r = search_dev("cmu440", 0, 9_999_999)
        ts.append(time.perf_counter() - t)
    return {"config1_ms": round(sorted(ts)[5] * 1e3, 3), "config1_result": list(r)}


def energy_meter(dev):
    """tools/energy.py's Meter for HIP device `dev` (amdsmi: the socket's energy counter and the
    firmware's limit accumulators), or None when the library cannot reach the device."""
    tools = os.path.join(ROOT, "tools")
    if tools not in sys.path:
        sys.path.insert(0, tools)
    try:
        import energy
        m = energy.meter_for_device(dev)
    except Exception as e:  # a missing amdsmi leaves the energy fields empty, not the line
        return {"error": f"{type(e).__name__}: {e}"}
    return m if m.ok else {"error": m.error}


def energy_fields(res, kc=None):
    """The line's energy object from a Window result (and the clock probe of the same search)."""
    if not res or "joules" not in res:
        return {"error": (res or {}).get("energy_error") or (res or {}).get("error") or "not measured"}
    snap = res.get("snapshot", {})
    out = {"j_per_gnonce": res.get("j_per_gnonce"), "mean_w": res.get("mean_w"),
           "kernel_clock_ghz": (kc or {}).get("ghz"), "joules": res["joules"], "seconds": res["seconds"],
           "nonces": res.get("nonces"), "limiter": res.get("limiter"),
           "limit_active_share": res.get("limit_active_share"),
           "power_limit_w": snap.get("power_limit_w"),
           # amdsmi reports N/A for these on the MI355X boxes measured so far: said, not left empty
           "gfx_voltage_mv": snap.get("voltage_gfx", "not exposed"),
           "socket_power_w": snap.get("current_socket_power"), "gfx_clk_mhz": snap.get("gfx_clk_mhz"),
           "throttle_status": snap.get("throttle_status", "not exposed"),
           "hotspot_c": snap.get("temperature_hotspot")}
    return out


def energy_total(per_device):
    """The timed region's energy over every device of the line, devices told apart by PCI address
    (ranks that share a device in a one-GPU rehearsal each read the whole device: the line then says
    so, and its joules count that device once per rank)."""
    rows = [p for p in per_device if (p.get("energy_timed") or {}).get("joules") is not None]
    if not rows:
        return None
    devs = {}
    for p in rows:
        devs.setdefault(p.get("pci") or p["dev"], []).append(p)
    joules = sum(p["energy_timed"]["joules"] for p in rows)
    nonces = sum(p["nonces"] for p in rows)
    sec = max(p["energy_timed"]["seconds"] for p in rows)
    return {"joules": round(joules, 2), "mean_w": round(joules / sec, 1) if sec else None,
            "j_per_gnonce": round(joules / (nonces / 1e9), 4) if nonces else None,
            "devices": len(devs), "shared_device": any(len(v) > 1 for v in devs.values()),
            "note": "socket energy counters (amdsmi) read just before and after the timed region, summed "
                    "over the devices of the line"}


def clock_search(msg, word, mode):
    """The un-profiled search the clock probe and the energy window run for a line whose dominant
    kernel is fast_search<word, mode>: the first decimal bucket of `msg` that holds 2^37 (else 2^36)
    nonces planned mostly on that layout, with a probe window that fits inside the search.  For
    "cmu440" and <4, One> (configs[1] and [3]) it is the d = 12 bucket from 10^11, kernel_clock's
    default.  None when no bucket qualifies (the caller keeps the default)."""
    import minehip
    for n, delay_s, window_s in ((1 << 37, 0.4, 1.2), (1 << 36, 0.3, 0.6)):
        for d in range(2, 21):
            lo = 10 ** (d - 1)
            top_of_bucket = 10 ** d - 1 if d < 20 else (1 << 64) - 1
            if lo + n - 1 > top_of_bucket:
                continue
            by_layout = {}
            for p in minehip.plan(msg, lo, lo + n - 1):
                if p["kind"] == 0:  # a bucket's launches are capped: sum them per layout
                    by_layout[(p["word"], p["mode"])] = by_layout.get((p["word"], p["mode"]), 0) + p["count"]
            if by_layout.get((word, mode), 0) * 2 >= n:
                return {"msg": msg, "lo": lo, "n": n, "delay_s": delay_s, "window_s": window_s}
    return None


def kernel_clock(search_dev, dev=0, delay_s=0.4, window_s=1.2, nwg=64, meter=None, msg="cmu440", lo=10 ** 11,
                 n=1 << 37):
    """The engine clock the fast kernel runs at, read inside the GPU during an un-profiled
    search (tools/clock_probe.hip, build/libclockprobe.so): one-wave probe workgroups on their
    own stream sleep through a 2^37-nonce search of the dominant layout (fast_search<4, One> at
    L = 3) and read the shader-clock and 100 MHz counters at both ends of a window inside it.
    Returns the median clock over the probes, the median per XCD and the search's own rate, or
    None when the probe library is missing or the window did not lie inside the search.
    With `meter` (energy_meter), the same search is bracketed by the socket's energy counter and
    the limit accumulators: the result's "energy" (J per 10^9 nonces, mean W, the active limit)."""
    import ctypes
    path = os.path.join(ROOT, "build", "libclockprobe.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.cp_start.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_int]
    lib.cp_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    # default: "cmu440" from 10^11, d = 12: last digit in word 4, the configs[1] d = 10 bucket's layout
    if lib.cp_start(dev, delay_s, window_s, nwg) != 0:
        return None
    buf = (ctypes.c_uint64 * (4 * nwg))()
    win = None
    if meter is not None and not isinstance(meter, dict):
        import energy
        win = energy.Window(meter, nonces=n, snap_after_s=delay_s + window_s / 2)
    try:
        t = time.perf_counter()
        if win is not None:
            with win:
                search_dev(msg, lo, lo + n - 1)
        else:
            search_dev(msg, lo, lo + n - 1)
        search_s = time.perf_counter() - t
    finally:
        rc = lib.cp_read(dev, buf, nwg)  # always: waits for the probes and frees their buffer
    if rc != 0:
        return None
    rows = [tuple(buf[4 * i:4 * i + 4]) for i in range(nwg)]
    ghz = [(x, c / (k / 1e8) / 1e9) for x, c, k, _ in rows if k]
    late = max(w for *_, w in rows) / 1e8  # window start after the workgroup started, s
    if not ghz or search_s < late + window_s + 0.1:
        out = {"ghz": None, "note": f"probe window not inside the search ({search_s:.2f} s)"}
        if win is not None:
            out["energy"] = energy_fields(win.result)
        return out

    def med(v):
        v = sorted(v)
        return v[len(v) // 2] if len(v) % 2 else (v[len(v) // 2 - 1] + v[len(v) // 2]) / 2

    by_xcd = {}
    for x, g in ghz:
        by_xcd.setdefault(int(x), []).append(g)
    out = {"ghz": round(med([g for _, g in ghz]), 4),
           "ghz_by_xcd": {str(x): round(med(v), 4) for x, v in sorted(by_xcd.items())},
           "probes": len(ghz), "window_s": window_s, "search_s": round(search_s, 3),
           "search_ghs": round(n / search_s / 1e9, 3),
           "search": {"msg_len": len(msg), "lo": lo, "nonces": n},
           "note": "s_memtime / s_memrealtime x 100 MHz in one-wave probe workgroups on their own stream, "
                   f"window {delay_s}..{delay_s + window_s} s into a {n}-nonce un-profiled search"
                   + (" of fast_search<4, One>" if (msg, lo) == ("cmu440", 10 ** 11) else f" from {lo}")
                   + " (tools/clock_probe.hip)"}
    if meter is not None:
        out["energy"] = (energy_fields(win.result, out) if win is not None else
                         {"error": meter.get("error", "no meter")})
    return out


def kernel_clocks(search_on, devices, probe=None, meters=None):
    """kernel_clock on every device at once, one host thread per device (the in-process N-GPU
    path): each device runs its own 2^37-nonce search with its probe inside,
    so the clocks are those of N devices under load together, as in the timed region.  With
    `meters` ({dev: energy_meter(dev)}) each device's search is also its energy window (VERDICT r05
    item 2: per-device power and J per 10^9 nonces beside the clock).
    search_on(dev) -> search_dev for that device.  Returns {dev: kernel_clock result or None}."""
    import threading
    probe = probe or kernel_clock
    out = {}

    def run(d):
        try:
            out[d] = (probe(search_on(d), d) if meters is None else
                      probe(search_on(d), d, meter=meters.get(d)))
        except Exception as e:  # a failed probe leaves that device's clock unknown, not the line
            out[d] = {"ghz": None, "note": f"probe failed: {e}"}

    th = [threading.Thread(target=run, args=(d,)) for d in sorted(set(devices))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out


def rank_device(local, ndev):
    """The HIP device of a launched rank: LOCAL_RANK when the process sees every GPU of the node,
    device 0 when the launcher gives each rank exactly one visible GPU (HIP/ROCR_VISIBLE_DEVICES
    per rank), None when LOCAL_RANK names no visible device."""
    if 0 <= local < ndev:
        return local
    if ndev == 1 and local >= 0:
        return 0
    return None


def ranks_per_device(idents):
    """The most ranks any one GPU serves, from every rank's device identity (PCI domain, bus,
    device): 1 on a node with a GPU per rank; more means the ranks share a card and per-GPU
    figures are not per-GPU (the one-GPU rehearsals set BENCH_DEVICE and expect it)."""
    from collections import Counter
    return max(Counter(tuple(i) for i in idents).values()) if idents else 0


N1_CHUNK_BITS = 32  # tests/golden/fullsize_cfg4.json: the minimum of every 2^32 chunk of configs[3]


def n1_slice(steps):
    """The configs[3] slice same_workload_n1 searches: the whole 2^32 chunks nearest to one step of
    K = max(steps, 20) (the driver's --steps 20 step: 12.8 chunks -> 13), from the chunk boundary
    at or below the middle step's start, so that tests/golden/fullsize_cfg4.json's chunk minima
    pin its result bit for bit."""
    k_all = max(steps, 20)
    k = k_all // 2
    s_lo, s_hi = step_range(CONFIGS["4"], k, k_all)
    c = 1 << N1_CHUNK_BITS
    n = max(1, round((s_hi - s_lo + 1) / c))
    lo = s_lo // c * c
    return lo, lo + n * c - 1, f"step {k} of {k_all}, rounded to {n} whole 2^{N1_CHUNK_BITS} chunks"


def same_workload_n1(search_dev, steps):
    """One step of the scaling workload on ONE device: BASELINE configs[3]'s middle slice
    ("cmu440", ~2^40 / K nonces with K = max(steps, 20): the driver's --steps 20 step, rounded to
    whole fixture chunks, n1_slice) searched alone.  The N > 1 lines run configs[3] and the N = 1
    line configs[1], so the driver's 1 -> N ratio would otherwise compare two workloads; every line
    carries this N = 1 figure of the same work (`n1_config4_ghs`) and, for configs[3] lines,
    value / (N x it) (`per_gpu_efficiency`).  Its result is checked against the fixture
    (`golden_ok`)."""
    cfg = CONFIGS["4"]
    lo, hi, what = n1_slice(steps)
    msg = cfg["msg"].encode()
    search_dev(msg, lo, lo + (1 << 30) - 1)  # untimed: device context, module and clocks up
    t = time.perf_counter()
    r = search_dev(msg, lo, hi)
    dt = time.perf_counter() - t
    expect = golden_expect(msg, lo, hi)
    return {"ghs": round((hi - lo + 1) / dt / 1e9, 4), "ms": round(dt * 1e3, 3), "range": [lo, hi],
            "slice": what, "result": list(r),
            "golden_ok": None if expect is None else tuple(r) == expect}


def per_gpu_efficiency(value, n_gpus, n1_ghs):
    """A line's whole-job GH/s over N x the one-device GH/s of the same workload."""
    return round(value / (n_gpus * n1_ghs), 4)


def power_sample(search_dev, dev=0, seconds=1.0):
    """amd-smi's socket power and GFX clocks sampled once while a ~1.5 s search runs (N = 1,
    after the timed region).  The kernel is VALU-bound at the package power limit, so power
    and clock are what differ between boxes.  None without amd-smi."""
    import re
    import threading
    smi = shutil.which("amd-smi")
    if not smi:
        return None
    t = threading.Thread(target=lambda: search_dev("cmu440", 10 ** 11, 10 ** 11 + (1 << 36) - 1))
    t.start()
    time.sleep(seconds)
    out = {}
    try:
        m = subprocess.run([smi, "metric", "--power", "--clock", "-g", str(dev)], capture_output=True,
                           text=True, timeout=20).stdout
        lim = subprocess.run([smi, "static", "--limit", "-g", str(dev)], capture_output=True, text=True,
                             timeout=20).stdout
    except (OSError, subprocess.TimeoutExpired):
        m, lim = "", ""
    t.join()
    for k, v in re.findall(r"(\w*POWER\w*):\s*([\d.]+)\s*W", m + "\n" + lim):
        out.setdefault(k.lower() + "_w", float(v))
    gfx = [float(v) for v in re.findall(r"GFX_\d+:\s*\n\s*CLK:\s*([\d.]+)\s*MHz", m)]
    if gfx:
        out["gfx_clk_mhz_mean"] = round(sum(gfx) / len(gfx), 1)
        out["gfx_clk_mhz"] = gfx
    out["note"] = "amd-smi metric/static, one sample during a 2^36-nonce search after the timed region"
    return out


def die(msg, code=2):
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)
    sys.exit(code)


def kernel_totals(per_dev_kstats):
    """Sum the per-(variant, lane length) HIP-event stats over devices; most algorithmic work
    (nonces x nonce_ops) first.  Not by time: with two streams a back-filling
    launch's HIP-event span includes its wait for free CUs, so its time overstates its share."""
    tot = {}
    for ks in per_dev_kstats:
        for k in ks:
            t = tot.setdefault((k["name"], k.get("lo_digits")),
                               dict(k, launches=0, nonces=0, ns=0, ops=0, slots=0))
            for f in ("launches", "nonces", "ns", "ops", "slots"):
                t[f] += k[f]
    return sorted(tot.values(), key=lambda k: -k["ops"])


def fast_loop_mix():
    """{(J, MODE): {"valu": N, "half": H}} of the per-nonce loops as built (build/fast_loop_mix.json,
    written by csrc/loop_mix.py from the assembly embedded in libminehip.so), or None."""
    try:
        with open(os.path.join(ROOT, "build", "fast_loop_mix.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return {tuple(int(x) for x in k.split(",")): v for k, v in d.items()}


def roofline(kst, cus, n_devices, resources=None, loop_mix=None):
    """Roofline of the dominant kernel from its HIP-event launch times (summed
    over devices, so achieved is per GPU).

    frac: the algorithm's per-nonce work over the VALU issue peak.  The work is
    nonce_ops (plan.cpp nonce_cost, exported per piece by mh_plan): the VALU
    instructions one nonce's SHA-256 needs once the rounds and schedule words
    shared by a lane's nonces are hoisted -- SURVEY §8(d) D4 restated for
    gfx950 (v_bitop3 xor3).  The kernel issues at least that many
    instructions per nonce (PMC SQ_INSTS_VALU: 1,200.6 for fast_search<4,0>
    against nonce_ops 1,195), so frac <= the hardware's issue fraction <= 1.
    frac_survey_d4 prices every nonce at SURVEY D4's 1,616 ops x tail blocks:
    a pricing convention that credits the hoisting and can exceed 1.

    mix_bound_frac: the most frac can reach -- a half-rate op never shares its
    quad-cycle with another half-rate op, so a nonce needs >= max(H, N/2)
    quad-cycles.  With loop_mix (fast_loop_mix()) H and N are those of the
    per-nonce loop as built (the add3 split trades half-rate ops for full-rate
    ones); alg_mix_bound_frac is the algorithm's own mix (nonce_slots)."""
    peak = cus * LANES_PER_CU_CLK * PEAK_SCLK_HZ / 1e12
    if not kst:
        return {"bound": "valu", "achieved": None, "peak": round(peak, 3), "frac": None}
    dom = kst[0]
    blocks = 1 if dom["mode"] % 3 == 0 else 2   # tail blocks hashed per nonce (Pre/Two and their Early modes: 2)
    sec = dom["ns"] * 1e-9
    nonces = max(1, dom["nonces"])
    ghs = dom["nonces"] / sec / 1e9
    ops = dom["ops"]                             # nonces x nonce_ops of every launch
    n_instr = ops / nonces
    n_half = (dom["slots"] - dom["ops"]) / nonces  # slots count a half-rate op twice
    achieved = ops / sec / 1e12
    alg_mix = n_instr / (2 * max(n_half, n_instr / 2))
    built = (loop_mix or {}).get((dom["word"], dom["mode"]))
    # the loop as built issues N' >= nonce_ops instructions, H' of them half rate
    mix = n_instr / (2 * max(built["half"], built["valu"] / 2)) if built else alg_mix
    d4 = dom["nonces"] * SURVEY_OPS_PER_COMPRESSION * blocks
    launches = max(1, dom["launches"])
    line = {
        "bound": "valu",
        "achieved": round(achieved, 3),
        "peak": round(peak, 3),
        "unit": "T int32 VALU lane-instructions/s per GPU",
        "frac": round(achieved / peak, 4),
        "frac_at_sclk": None,                    # against the peak at the clock the kernel ran at (PMC)
        # a kernel issues at least nonce_ops instructions per nonce, so frac > 1 would mean it skipped
        # work (or the HIP events mis-timed it): flagged, never hidden
        "frac_physical": achieved / peak <= 1.0,
        "basis": "algorithmic work per nonce = nonce_ops, the VALU instructions one nonce's SHA-256 "
                 "needs after hoisting the work a lane's nonces share (SURVEY §8(d) D4 restated for "
                 "gfx950, DESIGN.md §4), x the dominant kernel's nonces / its HIP-event launch time; "
                 f"peak = {cus} CU x 4 SIMD x 2 VALU instructions per quad-cycle x 64 lanes / 4 "
                 f"(= {LANES_PER_CU_CLK} lane-instructions/clk/CU) x {PEAK_SCLK_HZ / 1e9} GHz",
        "alg_instr_per_nonce": round(n_instr, 1),
        "half_rate_per_nonce": round(n_half, 1),
        # a half-rate op cannot share its quad-cycle with another half-rate op, so a nonce needs
        # >= max(H, N/2) quad-cycles: the most frac can reach with the loop as built
        "mix_bound_frac": round(mix, 4),
        "frac_of_mix_bound": round(achieved / peak / mix, 4),
        # the same bound for the algorithm's own mix (every add3 kept)
        "alg_mix_bound_frac": round(alg_mix, 4),
        "issued_loop": ({"valu_per_nonce": built["valu"], "half_rate_per_nonce": built["half"],
                         "source": "build/fast_loop_mix.json (csrc/loop_mix.py over the assembly embedded "
                                   "in libminehip.so)"} if built else None),
        "frac_survey_d4": round(d4 / sec / 1e12 / peak, 4),
        "frac_survey_d4_note": f"SURVEY §8(d) D4's {SURVEY_OPS_PER_COMPRESSION} ops per compression x "
                               f"{blocks} tail block(s) per nonce over the same time and peak: D4 prices "
                               "a nonce at full compressions, the kernel hoists what a lane's nonces "
                               "share, so this ratio credits the hoisting and can exceed 1",
        "kernel": dom["name"],
        "lo_digits": dom.get("lo_digits"),     # the launches' lane length (10^L nonces per lane)
        "tail_blocks": blocks,
        "launches": dom["launches"],
        "devices": n_devices,
        "avg_launch_ms": round(dom["ns"] / launches / 1e6, 4),
        "nonces_per_launch": dom["nonces"] // launches,
        "alg_instr_per_launch": ops // launches,
        "kernel_ghs": round(ghs, 4),
        "full_compression_instr": OPS_PER_BLOCK,
    }
    if resources:
        r = resources.get((dom["word"], dom["mode"]))
        if r:
            line["resources"] = dict(r, source="NT_AMDGPU_METADATA of the code object embedded in "
                                               "libminehip.so (minehip/codeobj.py)")
    if len(kst) > 1:
        s = kst[1]
        line["second_kernel"] = {"kernel": s["name"], "lo_digits": s.get("lo_digits"),
                                 "ms": round(s["ns"] / 1e6, 3),
                                 "kernel_ghs": round(s["nonces"] / (s["ns"] * 1e-9) / 1e9, 4),
                                 "alg_instr_per_nonce": round(s["ops"] / max(1, s["nonces"]), 1),
                                 "frac": round(s["ops"] / (s["ns"] * 1e-9) / 1e12 / peak, 4)}
        if resources and resources.get((s["word"], s["mode"])):
            line["second_kernel"]["resources"] = resources[(s["word"], s["mode"])]
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="workload (default: configs[1] '2' at N = 1, configs[3] '4' at N > 1)")
    ap.add_argument("--msg", default=None, help="override the config's message")
    ap.add_argument("--bits", type=int, default=None, help="override log2 nonces per GPU (weak) / total (strong)")
    ap.add_argument("--multi", action="store_true", help="N = 1 through mh_search_multi (the in-process path)")
    ap.add_argument("--devices", default=None,
                    help="in-process path: comma-separated device list (default 0..N-1); repeats rehearse "
                         "N workers on fewer GPUs, e.g. --gpus 4 --devices 0,0,0,0 on a 1-GPU box")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC passes")
    ap.add_argument("--no-clock", action="store_true",
                    help="skip the in-kernel clock probe after the timed region (tools/clock_probe.hip)")
    ap.add_argument("--no-n1", action="store_true",
                    help="skip the one-device search of a configs[3] step (n1_config4_ghs)")
    args = ap.parse_args()
    if args.gpus < 1 or args.steps < 1 or args.warmup < 0:
        die("--gpus and --steps must be >= 1, --warmup >= 0")
    cfg_name = args.config or default_config(args.gpus)
    cfg = dict(CONFIGS[cfg_name])
    if args.msg is not None:
        cfg["msg"] = args.msg
    if args.bits is not None:
        cfg["bits"] = args.bits

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    launched = world > 1
    if launched and world != args.gpus:
        die(f"--gpus {args.gpus} but WORLD_SIZE {world}: launch one process per GPU or none")
    # test-only: every rank on one device (rehearsing N > 1 on a 1-GPU box)
    if os.environ.get("BENCH_DEVICE") is not None:
        local = int(os.environ["BENCH_DEVICE"])

    # torch first: its HIP runtime must be the one loaded when libminehip's
    # dependency is resolved (the library then shares it).  device_count()
    # does not initialise the GPU.
    import torch
    ndev = torch.cuda.device_count()
    if launched:
        d = rank_device(local, ndev)
        if d is None:
            die(f"rank {rank}: HIP device {local} not visible ({ndev} visible)")
        devs = [d]
    elif args.devices:
        devs = [int(x) for x in args.devices.split(",")]
        if len(devs) != args.gpus or any(d < 0 or d >= ndev for d in devs):
            die(f"--devices {args.devices}: need {args.gpus} entries in [0, {ndev})")
    else:
        if ndev < args.gpus:
            die(f"--gpus {args.gpus} but {ndev} HIP device(s) visible")
        devs = list(range(args.gpus))
    torch.cuda.set_device(devs[0])
    import minehip
    if minehip.device_count() != ndev:
        die(f"libminehip sees {minehip.device_count()} devices, torch {ndev}")
    dist = None
    shared = None
    if launched:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)  # host merge: no RCCL
        pr = torch.cuda.get_device_properties(devs[0])
        idents = [None] * world
        dist.all_gather_object(idents, (pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id))
        shared = ranks_per_device(idents)
        if shared > 1 and os.environ.get("BENCH_DEVICE") is None and rank == 0:
            print(f"bench: {shared} ranks share one GPU (device visibility); per-GPU figures are not per GPU",
                  file=sys.stderr)

    msg = cfg["msg"].encode()
    n_gpus = args.gpus
    steps = args.steps
    multi = (not launched) and (n_gpus > 1 or args.multi)
    done = {d: 0 for d in devs}  # nonces searched per device in the timed region
    uniq = sorted(set(devs))

    # strong steps at N > 1: shards in proportion to each rank's measured rate (BENCH_BALANCE=0: equal)
    bal = Balancer(world, cfg["scaling"] == "strong" and os.environ.get("BENCH_BALANCE", "1") != "0")

    pipe = (LaunchedSteps(lambda a, b: minehip.search(msg, a, b, devs[0]), cfg, rank, world, steps, dist, bal)
            if launched else None)

    def step(k, timed=False):
        if launched:
            pipe.step(k)  # its host merge completes while the next step searches (LaunchedSteps)
            return None
        lo, hi = job_range(cfg, n_gpus, k, steps)
        if multi:
            return minehip.search_multi(msg, lo, hi, devs)
        return minehip.search(msg, lo, hi, devs[0])

    barrier = (lambda: dist.barrier()) if launched else (lambda: None)
    for w in range(args.warmup):
        step(w)
    if launched:
        pipe.finish()  # the warmup's merges (their rates size the timed shards)
        pipe.nonces = 0
    n1 = None
    if n_gpus > 1 and not args.no_n1:
        # the same workload on device 0 alone, before the timed region (the other ranks wait); the
        # first barrier lets every rank's warmup searches end first (on a one-GPU rehearsal they
        # would otherwise share rank 0's device during its search)
        barrier()
        if rank == 0:
            n1 = same_workload_n1(lambda m, a, b: minehip.search(m, a, b, devs[0]), steps)
        barrier()
    for d in uniq:
        minehip.profile_enable(d, True)
    # the energy of the timed region itself, per device of this process: counters read just outside
    # it (the window adds only the region's opening barrier and closing sync)
    meters = {d: energy_meter(d) for d in uniq}
    e_before = {d: m.read() for d, m in meters.items() if not isinstance(m, dict)}
    r, elapsed = run_timed(lambda k: step(k, timed=True), steps, 0, barrier, torch.cuda.synchronize,
                           finish=pipe.finish if launched else None)
    e_after = {d: meters[d].read() for d in e_before}
    if launched:
        done[devs[0]] += pipe.nonces
    per_dev = []
    for d in uniq:
        pr = minehip.profile_read(d)
        dp = torch.cuda.get_device_properties(d)
        per_dev.append({"dev": d, "rank": rank, "prof": pr, "kstats": minehip.profile_kernels(d),
                        # the physical GPU (a launched rank's device index is 0 when it sees one GPU)
                        "pci": f"{dp.pci_domain_id:04x}:{dp.pci_bus_id:02x}:{dp.pci_device_id:02x}"})
        minehip.profile_enable(d, False)
    for p in per_dev:
        p["nonces"] = done[p["dev"]] if launched else p["prof"]["fast_nonces"] + p["prof"]["generic_nonces"]
        p["elapsed"] = elapsed
        if p["dev"] in e_before:
            import energy
            w = energy.window_delta(e_before[p["dev"]], e_after[p["dev"]], p["nonces"])
            p["energy_timed"] = {k: w.get(k) for k in ("joules", "mean_w", "j_per_gnonce", "seconds", "limiter",
                                                        "energy_error")}
    if launched and not args.no_clock:
        # every rank's own GPU clock, read inside the GPU during an un-profiled search run by all
        # ranks at once after the timed region: what sets the per-GPU rates of a multi-GPU line;
        # the same search is the rank's energy window (socket power, J per 10^9 nonces, the limit)
        cs = (clock_search(cfg["msg"], per_dev[0]["kstats"][0]["word"], per_dev[0]["kstats"][0]["mode"])
              if per_dev and per_dev[0]["kstats"] else None) or {}
        kc = kernel_clock(lambda m, a, b: minehip.search(m, a, b, devs[0]), devs[0],
                          meter=energy_meter(devs[0]), **cs)
        for p in per_dev:
            p["kernel_clock_ghz"] = kc.get("ghz") if kc else None
            p["energy"] = kc.get("energy") if kc else None
    elif multi and not args.no_clock:
        # the in-process path: every device's clock and energy at once, one host thread per device
        kcs = kernel_clocks(lambda d: (lambda m, a, b: minehip.search(m, a, b, d)), uniq,
                            meters={d: energy_meter(d) for d in uniq})
        for p in per_dev:
            kc = kcs.get(p["dev"])
            p["kernel_clock_ghz"] = kc.get("ghz") if kc else None
            p["energy"] = kc.get("energy") if kc else None

    t_max = elapsed
    if launched:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t.item())
        gathered = [None] * world
        dist.all_gather_object(gathered, per_dev)
        per_dev = [p for g in gathered for p in g]

    if cfg["scaling"] == "weak":
        total = (1 << cfg["bits"]) * n_gpus * steps
        step_nonces = (1 << cfg["bits"]) * n_gpus
    else:
        total = 1 << cfg["bits"]
        step_nonces = total // steps
    value = total / t_max / 1e9
    props = torch.cuda.get_device_properties(devs[0])
    cus = int(props.multi_processor_count)
    kst = kernel_totals([p["kstats"] for p in per_dev])
    from minehip import codeobj
    roof = roofline(kst, cus, len(per_dev), codeobj.fast_kernel_resources(), fast_loop_mix())
    streams = 1 if os.environ.get("MINEHIP_STREAMS") == "1" else 2  # PlanOpts.streams (minehip.cpp plan_opts)
    roof["timing"] = {
        "source": "HIP events recorded around each fast launch on the stream it runs on (mh_profile_*)",
        "streams": streams,
        # with two streams an event span is a wall span: it includes any wait for CUs the other
        # stream's workgroups hold
        "wall_span": streams == 2,
        "note": "the dominant (full-L) launches go out first on the high-priority stream, so their spans "
                "are close to kernel time; tools/trace_frac.py recomputes frac from the rocprofv3 trace "
                "of the same command (per (kernel, queue) rows: profiles/*_kernel_stats_by_queue.csv)"
                if streams == 2 else "one stream: launches run one after another, spans are kernel times"}
    # the whole timed region on the same basis: every fast piece's nonces x nonce_ops over the
    # max-over-ranks wall time and all N GPUs' peak -- tails, generic edge launches, launch gaps,
    # the host merge and concurrent streams included (generic nonces, < 0.1%, not credited)
    all_ops = sum(p["prof"]["fast_ops"] for p in per_dev)
    roof["search_frac"] = round(all_ops / t_max / 1e12 / (n_gpus * roof["peak"]), 4)
    # algorithmic bytes of the dominant launch: one 16-byte (hash, nonce) partial per 256-lane workgroup
    job_lo, job_hi = job_range(cfg, n_gpus, 0, 1 if cfg["scaling"] == "weak" else steps)
    my_lo, my_hi = (rank_range(cfg, rank, world, 0, steps) if launched else (job_lo, job_hi))
    pieces = []
    for var in kst[:2]:
        # the PMC passes tell launches apart by kernel name only: a second variant that is the same
        # kernel at another lane length (e.g. a bucket's tail split) gets no PMC pass of its own
        if pieces and (var["word"], var["mode"]) == (pieces[0]["word"], pieces[0]["mode"]):
            break
        p = largest_piece(msg, my_lo, my_hi, var)
        if p is None:
            break
        pieces.append(p)
    if pieces:
        p = pieces[0]
        roof["algorithmic_bytes_per_launch"] = -(-(p["count"] // 10 ** p["lo_digits"]) // 256) * 16
    roof["traffic"] = None
    roof["traffic_note"] = "not measured (N > 1 or --no-pmc)"
    if rank == 0 and n_gpus == 1 and not args.no_pmc and pieces:
        vals, err = pmc_counters(cfg["msg"], pieces, devs[0])
        if vals is None:
            roof["traffic_note"] = err
        else:
            v0 = vals[f"fast_search<{pieces[0]['word']}, {pieces[0]['mode']}>"]
            # HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB, the 2x being gfx950's wide-read
            # correction (MI355X_MICROARCH.md, HBM section)
            roof["traffic"] = int((2 * v0["FETCH_SIZE"] + v0["WRITE_SIZE"]) * 1024)
            roof["traffic_unit"] = "bytes per launch (HBM, PMC)"
            roof["traffic_note"] = (f"FETCH_SIZE {v0['FETCH_SIZE']:.2f} KiB (x2 gfx950 correction), "
                                    f"WRITE_SIZE {v0['WRITE_SIZE']:.2f} KiB")
            roof["pmc"] = pmc_derived(v0, pieces[0], cus)
            roof["pmc"]["kernel"] = kst[0]["name"]
            # frac again against the peak at the clock this launch ran at
            at = roof["pmc"]["sclk_ghz"] * 1e9
            roof["frac_at_sclk"] = round(roof["achieved"] / (cus * LANES_PER_CU_CLK * at / 1e12), 4)
            roof["sclk_ghz"] = roof["pmc"]["sclk_ghz"]
            # what the hardware issued (PMC), against the same peak: >= frac, since the kernel issues
            # at least nonce_ops instructions per nonce
            roof["pmc"]["issued_frac_at_sclk"] = round(2 / roof["pmc"]["cycles_per_valu_instr"], 4)
            if len(pieces) > 1:
                v1 = vals[f"fast_search<{pieces[1]['word']}, {pieces[1]['mode']}>"]
                roof["second_kernel"]["pmc"] = pmc_derived(v1, pieces[1], cus)

    if rank == 0:
        # the merged range of the timed region
        m_lo = job_range(cfg, n_gpus, 0, steps)[0]
        m_hi = job_range(cfg, n_gpus, steps - 1, steps)[1]
        expect = golden_expect(msg, m_lo, m_hi)
        if n_gpus == 1 and not args.no_n1:
            n1 = same_workload_n1(lambda m, a, b: minehip.search(m, a, b, devs[0]), steps)
        cpu = None
        if n_gpus == 1 and not args.no_cpu_baseline:
            threads, facts = cpu_threads()
            cpu = cpu_baseline(cfg["msg"], threads)
            cpu.update(facts)
            # the shipped single-goroutine loop scales per core: what every visible core would do
            cpu["all_cores_estimate_ghs"] = round(cpu["single_thread_value"] * facts["cores_available"], 6)
            cpu["gpu_config1"] = gpu_config1(lambda m, a, b: minehip.search(m, a, b, devs[0]))
        if n_gpus == 1 and not launched and not args.no_pmc:
            roof["power"] = power_sample(lambda m, a, b: minehip.search(m, a, b, devs[0]), devs[0])
            if roof["power"] and roof["power"].get("gfx_clk_mhz_mean"):
                # amd-smi's clock of an un-profiled run reads at or above the in-kernel clock, the
                # PMC pass's (a profiled run) at or below it (MI355X_MICROARCH.md "DVFS give-back"):
                # the two fractions bracket the kernel's share of the peak at the clock it ran at
                smi = roof["power"]["gfx_clk_mhz_mean"] * 1e6
                roof["frac_at_smi_clk"] = round(roof["achieved"] / (cus * LANES_PER_CU_CLK * smi / 1e12), 4)
        if n_gpus == 1 and not launched and not args.no_clock:
            # the clock read inside the GPU during an un-profiled search of the same kernel, and the
            # fraction of the issue peak at that clock
            # the search is one of the dominant kernel's own layout (clock_search): configs[1]'s and
            # [3]'s is "cmu440" from 10^11; configs[2]'s lines get their messages' layouts
            cs = (clock_search(cfg["msg"], kst[0]["word"], kst[0]["mode"]) if kst else None) or {}
            kc = kernel_clock(lambda m, a, b: minehip.search(m, a, b, devs[0]), devs[0],
                              meter=energy_meter(devs[0]), **cs)
            if kc:
                # energy of the same un-profiled search: J per 10^9 nonces of
                # fast_search<4, One>, the socket's mean power, and which limit held the clock
                roof["energy"] = kc.pop("energy", None)
                roof["kernel_clock"] = kc
                if kc.get("ghz"):
                    at = kc["ghz"] * 1e9
                    roof["frac_at_kernel_clk"] = round(roof["achieved"] / (cus * LANES_PER_CU_CLK * at / 1e12), 4)
                    if roof.get("mix_bound_frac"):
                        roof["frac_of_mix_bound_at_kernel_clk"] = round(
                            roof["frac_at_kernel_clk"] / roof["mix_bound_frac"], 4)
        per_device = [{"dev": p["dev"], "rank": p["rank"], "nonces": p["nonces"],
                       "pci": p.get("pci"),
                       "ghs": round(p["nonces"] / p["elapsed"] / 1e9, 4),
                       "kernel_ghs": round(p["kstats"][0]["nonces"] / (p["kstats"][0]["ns"] * 1e-9) / 1e9, 4)
                       if p["kstats"] and p["kstats"][0]["ns"] else None,
                       "kernel_clock_ghz": p.get("kernel_clock_ghz"),
                       "energy": p.get("energy"), "energy_timed": p.get("energy_timed")}
                      for p in per_dev]
        if multi:  # the rates the library sized the last step's shards by (cost units per ns)
            for pd, rate in zip(per_device, minehip.multi_rates([p["dev"] for p in per_device])):
                pd["multi_rate"] = round(rate, 1)
        clocks = [p["kernel_clock_ghz"] for p in per_device if p.get("kernel_clock_ghz")]
        # per-device socket power and J per 10^9 nonces of the same concurrent search (N > 1): a node
        # power limit pulling the clocks down shows here, not as scheduling in per_gpu_efficiency
        watts = [p["energy"]["mean_w"] for p in per_device if (p.get("energy") or {}).get("mean_w")]
        jpg = [p["energy"]["j_per_gnonce"] for p in per_device if (p.get("energy") or {}).get("j_per_gnonce")]
        line = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "GH/s",
            "n_gpus": n_gpus,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / steps * 1e3, 3),
            # engine clock of the dominant kernel (PMC pass at N = 1; None otherwise): MI355X runs
            # this VALU-bound kernel at its package power limit, so the clock, and with it value,
            # differs from box to box
            "sclk_ghz": roof.get("sclk_ghz"),
            # the clock read inside the GPU during an un-profiled search of the dominant kernel (N = 1),
            # and value per GHz of it: the box-independent rate (boxes differ by their clock, §4)
            "kernel_clock_ghz": (roof.get("kernel_clock") or {}).get("ghz"),
            "ghs_per_kernel_ghz": (round(value / roof["kernel_clock"]["ghz"], 3)
                                   if (roof.get("kernel_clock") or {}).get("ghz") else None),
            # the scaling workload on one device (same_workload_n1): the N = 1 point of a configs[3]
            # curve, and this line's value against N times it when the line runs configs[3]
            "n1_config4_ghs": n1["ghs"] if n1 else None,
            # N > 1: the slowest and fastest device's in-kernel clock during a concurrent search after
            # the timed region -- with per_gpu_efficiency, whether a shortfall is clock spread between
            # power-limited devices or scheduling
            "kernel_clock_ghz_range": [min(clocks), max(clocks)] if n_gpus > 1 and clocks else None,
            "power_w_range": [min(watts), max(watts)] if n_gpus > 1 and watts else None,
            # the timed region's own energy, all devices: J per 10^9 nonces of the metric's workload
            # (every bucket of configs[1] at N = 1), from the socket counters read around it
            "energy_timed": energy_total(per_device),
            "j_per_gnonce_range": [min(jpg), max(jpg)] if n_gpus > 1 and jpg else None,
            "per_gpu_efficiency": (per_gpu_efficiency(value, n_gpus, n1["ghs"])
                                   if n1 and cfg_name == "4" and args.bits is None and args.msg is None else None),
            "n1_config4": n1,
            "higher_is_better": True,
            "scaling": cfg["scaling"],
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {
                "workload": cfg["desc"],
                "config": cfg_name,
                "msg": cfg["msg"] if len(cfg["msg"]) <= 16 else f"{cfg['msg'][:1]!r} x {len(cfg['msg'])}",
                "nonces_timed": total,
                "nonces_per_step": step_nonces,
                "nonces_per_gpu_per_step": step_nonces // n_gpus,
                "driver": ("one process per GPU (launcher), gloo host merge" if launched else
                           "one process, mh_search_multi: one host thread + HIP stream per device" if multi else
                           "one process, mh_search on one device"),
                "parallelism": f"contiguous shards over {n_gpus} GPU(s), 16-byte (hash, nonce) host merge, no RCCL",
                # in-process: the device of every worker (a repeat rehearses N workers on fewer GPUs)
                "devices": devs if multi else None,
                # launched: the most ranks one physical GPU served (1 = one GPU per rank)
                "ranks_per_device": shared if launched else None,
                "shards": ("each strong step split in proportion to every rank's measured search rate "
                           "(gathered with the host merges of the steps before the last, which run while "
                           "the next step searches)" if launched and bal.enabled else
                           "one shard per device per step, sized by each device's rate measured on the earlier "
                           "steps (mh_search_multi)" if multi else "equal"),
            },
            "per_device": per_device,
            "roofline": roof,
            "cpu_baseline": cpu,
            # self-check on the product path: the winning nonce re-hashed by the
            # generic kernel (mh_hash_batch), not the fast kernel that found it
            "result": {"hash": r[0], "nonce": r[1],
                       "rehash_ok": minehip.Hash(msg, r[1], devs[0]) == r[0],
                       "range": [m_lo, m_hi],
                       # bit-exact against the full-size fixture when one covers the range
                       "golden_ok": None if expect is None else tuple(r) == expect},
        }
        print(json.dumps(line), flush=True)
    if launched:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
