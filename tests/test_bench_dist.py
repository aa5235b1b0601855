"""bench.py's multi-GPU logic on CPU.

* The launched path (one process per GPU) over gloo at world 2 and 3: each
  rank scans its shard of every step, the 16-byte (hash, nonce) tuples are
  merged on the host (gloo all_gather of CPU tensors, no RCCL), and the
  max-over-ranks time is agreed.  The per-rank search is the oracle here (no
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


def _worker(rank, world, port, cfg, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = []

    def step(k):
        rr = bench.rank_range(cfg, rank, world, k, steps)
        mine.append(rr)
        r = oracle.search(MSG, rr[0], rr[1]) if rr else ((1 << 64) - 1, (1 << 64) - 1)
        return bench.host_merge(r, world, dist)

    r, elapsed = bench.run_timed(step, steps, 1, dist.barrier, lambda: None)
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, r, float(t.item()), mine[1:]))  # mine[0] is the warmup step
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,scaling", [(2, "strong"), (3, "strong"), (2, "weak")])
def test_sharded_merge_matches_full_scan(world, scaling):
    bits, steps = (15, 4) if scaling == "strong" else (12, 2)
    cfg = dict(msg="cmu440", bits=bits, scaling=scaling)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lo, hi = 0, ((1 << bits) if scaling == "strong" else world << bits) - 1
    exp = oracle.search(MSG, lo, hi)
    assert all(o[1] == exp for o in out)          # every rank holds the merged min of the job
    assert len({o[2] for o in out}) == 1          # max-over-ranks time agreed
    if scaling == "strong":                       # the timed steps covered [lo, hi] exactly once
        rs = sorted(r for o in out for r in o[3])
        assert rs[0][0] == lo and rs[-1][1] == hi
        assert all(rs[i][1] + 1 == rs[i + 1][0] for i in range(len(rs) - 1))


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
