"""bench.py's multi-GPU logic on CPU.

* The launched path (one process per GPU) over gloo at world 2 and 3: each
  rank scans its shard of every step, the 16-byte (hash, nonce) tuples are
  merged on the host (gloo all_gather of CPU tensors, no RCCL; each step's
  merge posted asynchronously and completed while the next step searches,
  bench.LaunchedSteps), and the max-over-ranks time is agreed.  The per-rank search is the oracle here (no
  GPU); on the box it is minehip.search.
* Workload tiling: configs[3]'s K strong steps x N shards cover [0, 2^40-1]
  exactly once; weak shards tile [0, N*2^32).
* The CLI contract: `--gpus N` with fewer than N visible devices, or a
  launcher whose WORLD_SIZE differs from --gpus, exits 2 with no JSON line.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MSG = b"cmu440"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, steps, q, balance=False, slow_ns=0, warmup=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = []
    bal = bench.Balancer(world, balance)

    def search(a, b):
        mine.append((a, b))
        r = oracle.search(MSG, a, b)
        if slow_ns:  # a slower device: rank r takes (r + 1) x slow_ns per nonce
            time.sleep((b - a + 1) * slow_ns * (rank + 1) * 1e-9)
        return r

    pipe = bench.LaunchedSteps(search, cfg, rank, world, steps, dist, bal)
    r, elapsed = bench.run_timed(pipe.step, steps, warmup, dist.barrier, lambda: None, finish=pipe.finish)
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, r, float(t.item()), mine[warmup:], bal.weights()))  # mine[:warmup]: the warmup steps
    dist.barrier()
    dist.destroy_process_group()


def _launch(world, cfg, steps, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, steps, q), kwargs=kw) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _tiles_once(out, lo, hi):
    rs = sorted(r for o in out for r in o[3])
    return rs[0][0] == lo and rs[-1][1] == hi and all(rs[i][1] + 1 == rs[i + 1][0] for i in range(len(rs) - 1))


@pytest.mark.parametrize("world,scaling", [(2, "strong"), (3, "strong"), (2, "weak")])
def test_sharded_merge_matches_full_scan(world, scaling):
    bits, steps = (15, 4) if scaling == "strong" else (12, 2)
    cfg = dict(msg="cmu440", bits=bits, scaling=scaling)
    out = _launch(world, cfg, steps)
    lo, hi = 0, ((1 << bits) if scaling == "strong" else world << bits) - 1
    exp = oracle.search(MSG, lo, hi)
    assert all(o[1] == exp for o in out)          # every rank holds the merged min of the job
    assert len({o[2] for o in out}) == 1          # max-over-ranks time agreed
    if scaling == "strong":                       # the timed steps covered [lo, hi] exactly once
        assert _tiles_once(out, lo, hi)


def test_balanced_strong_shards_follow_rates():
    """bench.py's default at N > 1 (strong steps): shards in proportion to each rank's measured
    rate.  Rank 1 is made 2x slower per nonce; after the warmup steps it gets about a third of
    every step, every rank computes the same weights, the timed steps still tile the job once
    and the merged result is the full scan's."""
    world, bits, steps = 2, 16, 4
    cfg = dict(msg="cmu440", bits=bits, scaling="strong")
    out = _launch(world, cfg, steps, balance=True, slow_ns=10000, warmup=3)  # sleeps >> scheduling noise
    lo, hi = 0, (1 << bits) - 1
    assert all(o[1] == oracle.search(MSG, lo, hi) for o in out)
    assert _tiles_once(out, lo, hi)
    assert out[0][4] == out[1][4] and out[0][4] is not None      # same weights on every rank
    last = [o[3][-1][1] - o[3][-1][0] + 1 for o in out]          # each rank's share of the last step
    assert 0.25 < last[1] / sum(last) < 0.42, last


@pytest.mark.parametrize("world", [2, 3, 8])
def test_weighted_split_tiles(world):
    for weights in ([1] * world, list(range(1, world + 1)), [1 << 20] + [1] * (world - 1)):
        for lo, hi in ((0, 99), (5, 5 + 10 ** 9), (0, (1 << 40) - 1)):
            rs = [bench.weighted_split(lo, hi, weights, i) for i in range(world)]
            rs = [r for r in rs if r]
            assert rs[0][0] == lo and rs[-1][1] == hi
            assert all(rs[i][1] + 1 == rs[i + 1][0] for i in range(len(rs) - 1))
    assert bench.weighted_split(0, 99, [1, 3], 0) == (0, 24)
    assert bench.weighted_split(0, 99, [1, 3], 1) == (25, 99)


def test_balancer_skips_the_first_step_and_needs_every_rate():
    b = bench.Balancer(2)
    b.update([(100, 10 ** 9), (100, 10 ** 9)])   # first step: context / module load, not counted
    assert b.weights() is None
    b.update([(100, 1000), (0, 1000)])             # a rank without nonces: no rate yet
    assert b.weights() is None
    b.update([(100, 1000), (300, 1000)])             # cumulative: 200 / 2000 ns against 300 / 2000 ns
    assert b.weights() == [round(bench.Balancer.SCALE * 2 / 3), bench.Balancer.SCALE]
    assert bench.Balancer(2, enabled=False).weights() is None
    assert bench.Balancer(1).weights() is None


def test_merge_is_lexicographic():
    assert bench.merge([(5, 9), (5, 3), (7, 1)]) == (5, 3)
    assert bench.shard(3, 32) == (3 << 32, (4 << 32) - 1)


def test_host_merge_keeps_u64_order():
    """The u64 -> i64 shift used for the gloo tensors keeps the order of values >= 2^63."""
    vals = [(0, 5), ((1 << 63) - 1, 1), (1 << 63, 0), ((1 << 64) - 1, (1 << 64) - 1)]
    for a in vals:
        enc = (a[0] - (1 << 63), a[1] - (1 << 63))
        assert all(-(1 << 63) <= v < (1 << 63) for v in enc)
        assert tuple(v + (1 << 63) for v in enc) == a
    assert sorted(vals, key=lambda a: (a[0] - (1 << 63), a[1] - (1 << 63))) == sorted(vals)


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("steps", [1, 5, 20, 7])
def test_strong_steps_tile_config3_once(world, steps):
    cfg = bench.CONFIGS["4"]
    rs = [bench.rank_range(cfg, r, world, k, steps) for k in range(steps) for r in range(world)]
    rs = sorted(r for r in rs if r)
    assert rs[0][0] == 0 and rs[-1][1] == (1 << 40) - 1
    assert all(rs[i][1] + 1 == rs[i + 1][0] for i in range(len(rs) - 1))
    sizes = [b - a + 1 for a, b in rs]
    assert max(sizes) - min(sizes) <= 1           # equal shards: no rank waits on another
    assert bench.job_range(cfg, world, 0, steps)[0] == 0
    assert bench.job_range(cfg, world, steps - 1, steps)[1] == (1 << 40) - 1


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_weak_shards_tile(world):
    cfg = bench.CONFIGS["2"]
    rs = [bench.rank_range(cfg, r, world) for r in range(world)]
    assert rs[0][0] == 0 and all(rs[i][1] + 1 == rs[i + 1][0] for i in range(world - 1))
    assert rs[-1][1] == (world << 32) - 1 == bench.job_range(cfg, world)[1]


def test_default_workloads():
    assert bench.default_config(1) == "2"       # configs[1], the metric's single-GPU config
    for n in (2, 4, 8):
        assert bench.default_config(n) == "4"   # configs[3], the scaling curve


def test_golden_expect_covers_every_bench_range():
    """bench.py's result.golden_ok lookup: configs[1] at N = 1 and the weak shards at N = 2, 4, 8,
    configs[2] at N = 1 come from the full-size fixtures; ranges no fixture covers give None,
    never an exception."""
    for world in (1, 2, 4, 8):
        lo, hi = bench.job_range(bench.CONFIGS["2"], world)
        assert bench.golden_expect(MSG, lo, hi) is not None, world
    assert bench.golden_expect(MSG, 0, (1 << 32) - 1) == (3580905509, 4025695320)
    for cfg in ("3a", "3b"):
        c = bench.CONFIGS[cfg]
        assert bench.golden_expect(c["msg"].encode(), 0, (1 << c["bits"]) - 1) is not None
    assert bench.golden_expect(b"no fixture", 0, 99) is None
    assert bench.golden_expect(MSG, 5, 1 << 33) is None  # not chunk-aligned
    # the N > 1 default (configs[3], strong): the timed region's merged range is [0, 2^40-1],
    # answered by the whole-range fixture, so the driver's 2/4/8-GPU lines carry golden_ok
    c4 = bench.CONFIGS["4"]
    for world in (2, 4, 8):
        lo = bench.job_range(c4, world, 0, 20)[0]
        hi = bench.job_range(c4, world, 19, 20)[1]
        assert (lo, hi) == (0, (1 << 40) - 1)
        assert bench.golden_expect(MSG, lo, hi) == (26475375, 32018601659), world


def _run_bench(args, env_extra=None):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "BENCH_DEVICE"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args, "--no-pmc",
                           "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=300)


def _json_lines(out):
    lines = []
    for ln in out.splitlines():
        try:
            lines.append(json.loads(ln))
        except ValueError:
            pass
    return lines


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is None and os.path.exists("/dev/kfd"),
                    reason="a GPU may be visible: the device-count refusal is only checked without one")
@pytest.mark.parametrize("gpus", [1, 2, 8])
def test_too_few_devices_exits_without_json(gpus):
    p = _run_bench(["--gpus", str(gpus), "--steps", "1", "--warmup", "0"])
    assert p.returncode == 2, p.stderr
    assert "device" in p.stderr
    assert _json_lines(p.stdout) == []


def test_world_size_mismatch_exits_without_json():
    p = _run_bench(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2, p.stderr
    assert "WORLD_SIZE" in p.stderr
    assert _json_lines(p.stdout) == []


def test_rank_device_and_sharing():
    """A launched rank runs on LOCAL_RANK when it sees the node's GPUs, on device 0 when the
    launcher isolates one GPU per rank, and refuses a LOCAL_RANK naming no device; the line's
    ranks_per_device counts ranks per physical GPU (PCI identity)."""
    assert bench.rank_device(3, 8) == 3
    assert bench.rank_device(0, 8) == 0
    assert bench.rank_device(5, 1) == 0    # HIP/ROCR_VISIBLE_DEVICES per rank
    assert bench.rank_device(5, 4) is None
    assert bench.rank_device(0, 0) is None
    assert bench.ranks_per_device([(0, 0x11, 0), (0, 0x21, 0), (0, 0x31, 0)]) == 1
    assert bench.ranks_per_device([(0, 0x11, 0)] * 8) == 8     # the one-GPU rehearsal
    assert bench.ranks_per_device([(0, 0x11, 0), (0, 0x11, 0), (0, 0x21, 0)]) == 2


def test_same_workload_n1_slice_and_efficiency():
    """Every line's n1_config4_ghs is one configs[3] step -- the middle 2^40/20 slice the driver's
    --steps 20 line runs, rounded to whole 2^32 fixture chunks -- searched on one device;
    per_gpu_efficiency = value / (N x it).  Its result is pinned by
    fullsize_cfg4.json's chunk minima (golden_ok, not null).  The search here
    is a stub (no GPU) that returns the fixture's answer for the slice."""
    calls = []

    def search(m, a, b):
        calls.append((m, a, b))
        time.sleep(0.01)
        return bench.golden_expect(m, a, b) or (1, a)

    r = bench.same_workload_n1(search, 20)
    lo, hi = 1 << 39, (1 << 39) + 13 * (1 << 32) - 1     # step 10 of 20 starts at 2^39; 12.8 -> 13 chunks
    s_lo, s_hi = bench.step_range(bench.CONFIGS["4"], 10, 20)
    assert s_lo == lo and abs((hi - lo + 1) / (s_hi - s_lo + 1) - 1) < 0.02
    assert calls[-1] == (b"cmu440", lo, hi) and r["range"] == [lo, hi]
    assert calls[0][1] == lo and calls[0][2] < hi       # the untimed warm-up search comes first
    assert 0 < r["ghs"] < (hi - lo + 1) / 0.01 / 1e9 * 1.0001
    assert r["slice"].startswith("step 10 of 20")
    assert bench.golden_expect(b"cmu440", lo, hi) is not None and r["golden_ok"] is True
    assert bench.same_workload_n1(lambda m, a, b: (0, a), 20)["golden_ok"] is False
    # fewer steps than the driver's: the driver's step; more: the middle step of those, still whole chunks
    assert bench.same_workload_n1(search, 5)["range"] == [lo, hi]
    r40 = bench.same_workload_n1(search, 40)
    assert r40["range"] == [lo, lo + 6 * (1 << 32) - 1] and r40["golden_ok"] is True
    assert bench.per_gpu_efficiency(430.0, 8, 54.0) == round(430.0 / 432.0, 4)
    assert bench.per_gpu_efficiency(54.0, 1, 54.0) == 1.0


def test_cpu_baseline_threads(monkeypatch):
    """The CPU baseline runs on every core of the affinity mask unless a cgroup quota or the job's
    CPU share (OMP_NUM_THREADS, which the GPU box sets per one-GPU job) is smaller, and says
    which; BENCH_CPU_THREADS overrides."""
    avail = len(os.sched_getaffinity(0))
    monkeypatch.delenv("BENCH_CPU_THREADS", raising=False)
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: None)
    t, f = bench.cpu_threads()
    assert t == avail == f["cores_available"] and f["cores_rule"] == "every core in the affinity mask"
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    t, f = bench.cpu_threads()
    assert t == 1 and f["job_cpu_share"] == 1 and f["cores_available"] == avail
    monkeypatch.setenv("OMP_NUM_THREADS", str(avail + 64))
    assert bench.cpu_threads()[0] == avail
    monkeypatch.setattr(bench, "cgroup_cpu_quota", lambda: 1)
    t, f = bench.cpu_threads()
    assert t == 1 and f["cgroup_quota_cores"] == 1
    monkeypatch.setenv("BENCH_CPU_THREADS", "3")
    assert bench.cpu_threads()[0] == 3


# ---- the driver's N > 1 commands, on the one GPU of a test box ----------
# The driver's scaling run is `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`
# (or `python bench.py --gpus N` in one process) on an 8-GPU node, once per round; a bench-only
# regression there (r04a's TypeError in the in-process line) would cost the only 8-GPU curve.  Both
# paths run here as fresh child processes with two workers on device 0, on configs[3] cut to
# [0, 2^35 - 1] (fullsize_cfg2.json pins its answer), and must print one good JSON line.

BENCH_N2 = ["--config", "4", "--bits", "35", "--steps", "4", "--warmup", "1", "--no-pmc", "--no-cpu-baseline"]


def _run_group(cmd, env, timeout):
    """Run cmd in its own process group; on a time limit kill the whole group (the launcher's ranks
    included) and fail."""
    import signal
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        pytest.fail(f"{' '.join(cmd[:4])}... timed out after {timeout} s\n{err[-3000:]}")
    return p.returncode, out, err


def _skip_without_energy_counter(e):
    """A box whose amdsmi cannot reach the GPU's energy counter (never seen on the MI355X pool) makes
    the line say so in place of the numbers; that is the plumbing working, not a failure."""
    if e and "error" in e and "mean_w" not in e:
        pytest.skip(f"energy counter not available on this box: {e['error']}")


def _check_n2_line(line, driver):
    assert line["n_gpus"] == 2 and line["steps"] == 4 and line["value"] > 0
    assert line["config"]["config"] == "4" and driver in line["config"]["driver"]
    assert line["result"]["range"] == [0, (1 << 35) - 1]
    assert line["result"]["golden_ok"] is True and line["result"]["rehash_ok"] is True
    assert line["n1_config4"] and line["n1_config4"]["golden_ok"] is True and line["n1_config4_ghs"] > 0
    assert line["per_gpu_efficiency"] is None  # --bits: not configs[3] as the driver runs it
    assert line["roofline"]["frac"] and 0 < line["roofline"]["frac"] <= 1
    for p in line["per_device"]:
        assert p["dev"] == 0 and p["nonces"] > 0 and p["kernel_clock_ghz"] and 1.0 < p["kernel_clock_ghz"] <= 2.5, p
        # each device's socket power and J per 10^9 nonces of the same
        # concurrent search, and the limit that held its clock
        e = p["energy"]
        _skip_without_energy_counter(e)
        assert e and 100 < e["mean_w"] < 2000 and 5 < e["j_per_gnonce"] < 200, e
        assert e["kernel_clock_ghz"] == p["kernel_clock_ghz"] and e["limiter"], e
    lo, hi = line["kernel_clock_ghz_range"]
    assert 1.0 < lo <= hi <= 2.5
    wlo, whi = line["power_w_range"]
    jlo, jhi = line["j_per_gnonce_range"]
    assert 100 < wlo <= whi < 2000 and 5 < jlo <= jhi < 200


@pytest.mark.gpu
def test_bench_inprocess_two_workers_one_gpu():
    """`python bench.py --gpus 2 --devices 0,0`: the in-process path (mh_search_multi, one host
    thread per worker) with both workers on device 0; per_device has one entry per distinct device,
    carrying its in-kernel clock read during a concurrent search."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "BENCH_DEVICE"):
        env.pop(k, None)
    rc, out, err = _run_group([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2",
                               "--devices", "0,0", *BENCH_N2], env, 200)
    assert rc == 0, err[-3000:]
    lines = _json_lines(out)
    assert len(lines) == 1, out[-2000:]
    line = lines[0]
    _check_n2_line(line, "mh_search_multi")
    assert line["config"]["devices"] == [0, 0] and len(line["per_device"]) == 1
    assert line["per_device"][0]["nonces"] == 1 << 35


@pytest.mark.gpu
def test_bench_launched_two_ranks_one_gpu():
    """`torch.distributed.run --nproc-per-node 2 bench.py --gpus 2` (the driver's form) with both
    ranks on device 0 (BENCH_DEVICE=0): the gloo host merge, the rate-balanced strong shards, two
    per_device entries (one per rank, each with its clock) and ranks_per_device 2."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    rc, out, err = _run_group([sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1",
                               "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", str(port),
                               os.path.join(ROOT, "bench.py"), "--gpus", "2", *BENCH_N2], env, 240)
    assert rc == 0, err[-3000:]
    lines = _json_lines(out)
    assert len(lines) == 1, out[-2000:]
    line = lines[0]
    _check_n2_line(line, "one process per GPU")
    assert sorted(p["rank"] for p in line["per_device"]) == [0, 1]
    assert sum(p["nonces"] for p in line["per_device"]) == 1 << 35
    assert line["config"]["ranks_per_device"] == 2


@pytest.mark.gpu
def test_bench_one_gpu_line_carries_energy():
    """`python bench.py` at N = 1 (short): the line names the energy of the clock probe's search
    (`roofline.energy`: J per 10^9 nonces, mean W, the active limit, the power limit, "not exposed"
    where amdsmi has nothing) and of the timed region itself (`energy_timed`), for one device known
    by its PCI address."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "BENCH_DEVICE"):
        env.pop(k, None)
    rc, out, err = _run_group([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                               "--no-pmc", "--no-cpu-baseline", "--no-n1"], env, 200)
    assert rc == 0, err[-3000:]
    lines = _json_lines(out)
    assert len(lines) == 1, out[-2000:]
    line = lines[0]
    assert line["result"]["golden_ok"] is True
    e = line["roofline"]["energy"]
    _skip_without_energy_counter(e)
    assert 100 < e["mean_w"] < 2000 and 5 < e["j_per_gnonce"] < 200 and e["limiter"], e
    assert e["kernel_clock_ghz"] == line["kernel_clock_ghz"] and e["power_limit_w"], e
    assert set(e["limit_active_share"]) >= {"ppt_pwr", "socket_thrm", "vr_thrm", "hbm_thrm", "prochot_thrm"}, e
    assert e["gfx_voltage_mv"] is not None and e["throttle_status"] is not None  # a value or "not exposed"
    t = line["energy_timed"]
    assert t and t["devices"] == 1 and t["shared_device"] is False and 5 < t["j_per_gnonce"] < 200, t
    assert line["per_device"][0]["pci"] and line["per_device"][0]["energy_timed"]["joules"] > 0
