"""The multi-GPU path of bench.py on CPU: world_size 2 over gloo, each rank
scanning its own shard (weak scaling, no data-path collective), the 16-byte
(hash, nonce) tuples merged by all_gather.  The per-rank search is the oracle
here (no GPU); on the box it is minehip.search."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from oracle import oracle

BITS = 13
MSG = b"cmu440"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = bench.shard(rank, BITS)
    r, elapsed = bench.run_steps(lambda a, b: oracle.search(MSG, a, b), lo, hi, steps=2, warmup=1,
                                 world=world, dist=dist, torch=torch, device=torch.device("cpu"),
                                 sync=lambda: None)
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put((rank, r, float(t.item()), (lo, hi)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_merge_matches_full_scan(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    shards = sorted(o[3] for o in out)
    assert shards[0][0] == 0 and all(shards[i][1] + 1 == shards[i + 1][0] for i in range(world - 1))
    exp = oracle.search(MSG, 0, world * (1 << BITS) - 1)
    assert all(o[1] == exp for o in out)          # every rank holds the merged min
    assert len({o[2] for o in out}) == 1          # max-over-ranks time agreed


def test_merge_is_lexicographic():
    assert bench.merge([(5, 9), (5, 3), (7, 1)]) == (5, 3)
    assert bench.shard(3, 32) == (3 << 32, (4 << 32) - 1)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rank_ranges_tile_the_space(world):
    for bits, scaling in ((32, "weak"), (40, "strong"), (7, "strong")):
        rs = [bench.rank_range(r, world, bits, scaling) for r in range(world)]
        assert rs[0][0] == 0 and all(rs[i][1] + 1 == rs[i + 1][0] for i in range(world - 1))
        total = (1 << bits) * (world if scaling == "weak" else 1)
        assert rs[-1][1] == total - 1


def test_golden_expect_covers_every_bench_range():
    """bench.py's result.golden_ok lookup: the merged range of configs[1] at N = 1, 2, 4, 8 and of
    configs[2] at N = 1 come from the full-size fixtures; ranges no fixture covers give None
    (configs[3]: 2^40), never an exception."""
    for world in (1, 2, 4, 8):
        lo = min(bench.rank_range(r, world, 32, "weak")[0] for r in range(world))
        hi = max(bench.rank_range(r, world, 32, "weak")[1] for r in range(world))
        assert bench.golden_expect(MSG, lo, hi) is not None, world
    assert bench.golden_expect(MSG, 0, (1 << 32) - 1) == (3580905509, 4025695320)
    for cfg in ("3a", "3b"):
        c = bench.CONFIGS[cfg]
        assert bench.golden_expect(c["msg"].encode(), 0, (1 << c["bits"]) - 1) is not None
    assert bench.golden_expect(MSG, 0, (1 << 40) - 1) is None
    assert bench.golden_expect(b"no fixture", 0, 99) is None
