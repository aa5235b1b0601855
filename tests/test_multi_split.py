"""CPU tests of mh_search_multi's adaptive split (chunk = 0), through the host-only
mh_multi_plan: one contiguous head shard per device, sized by the device's rate in cost units,
plus a dynamic tail on long ranges.  The spans must
tile the request range exactly once, whatever the weights, so the merged (hash, nonce) cannot
depend on the split (the GPU tests check the result itself)."""
import random

import pytest

import minehip

U64 = (1 << 64) - 1
TAIL_MIN_PER_WORKER = 1 << 35  # minehip.cpp kTailMinPerWorker


def check_tiles(spans, lo, hi):
    cur = lo
    for s in sorted(spans, key=lambda s: s["lower"]):
        assert s["lower"] == cur and s["upper"] >= s["lower"], (s, cur)
        cur = s["upper"] + 1
    assert cur - 1 == hi


def test_split_tiles_exactly():
    rng = random.Random(440)
    msgs = [b"cmu440", b"x" * 60, b"a" * 100, b""]
    for _ in range(300):
        m = rng.choice(msgs)
        n = rng.randrange(1, 9)
        k = rng.randrange(0, 20)
        lo = rng.randrange(0, 10 ** k + 1)
        hi = min(U64, lo + rng.choice([0, 1, 7, rng.randrange(0, 1 << rng.randrange(1, 64))]))
        w = None if rng.random() < 0.3 else [rng.uniform(0.5, 2.0) for _ in range(n)]
        spans = minehip.multi_plan(m, lo, hi, n, w)
        check_tiles(spans, lo, hi)
        heads = [s for s in spans if s["kind"] == 0]
        assert [s["worker"] for s in heads] == sorted(s["worker"] for s in heads)  # worker order
        assert len({s["worker"] for s in heads}) == len(heads) <= n
        assert all(s["worker"] == -1 for s in spans if s["kind"] == 1)
    for lo, hi in ((0, U64), (U64, U64), (U64 - 5, U64), (0, 0)):
        for n in (1, 3, 8):
            check_tiles(minehip.multi_plan(b"cmu440", lo, hi, n), lo, hi)


def test_heads_follow_weights_by_cost():
    """Shards carry cost in proportion to the weights (the device rates), to within one nonce's
    cost; the shard holding configs[3]'s small buckets (d <= 10: shorter lanes, generic edges) gets
    fewer nonces for the same cost."""
    lo, hi = 0, (1 << 40) // 20 - 1  # one step of the bench's configs[3] line
    w = [1.0, 1.05, 0.97, 1.0, 1.0, 1.02, 0.99, 1.0]
    spans = minehip.multi_plan(b"cmu440", lo, hi, 8, w)
    assert [s["kind"] for s in spans] == [0] * 8  # 6.9e9 nonces per worker: no tail
    tot = sum(s["cost"] for s in spans)
    for s in spans:
        assert s["cost"] / tot == pytest.approx(w[s["worker"]] / sum(w), rel=1e-6)
    eq = minehip.multi_plan(b"cmu440", lo, hi, 8)
    sizes = [s["upper"] - s["lower"] + 1 for s in eq]
    assert sizes[0] < min(sizes[1:])
    assert max(sizes[1:]) - min(sizes[1:]) <= 2


def test_dynamic_tail_on_long_ranges():
    """>= 2^35 nonces per worker: the last 1/16 of the cost goes out as 2 chunks per worker, handed
    to whichever worker finishes first; below that every worker runs exactly one search."""
    for n in (2, 4, 8):
        hi = n * TAIL_MIN_PER_WORKER - 1
        spans = minehip.multi_plan(b"cmu440", 0, hi, n)
        tail = [s for s in spans if s["kind"] == 1]
        assert len(tail) == 2 * n
        tot = sum(s["cost"] for s in spans)
        assert sum(s["cost"] for s in tail) / tot == pytest.approx(1 / 16, rel=1e-6)
        assert min(s["lower"] for s in tail) > max(s["upper"] for s in spans if s["kind"] == 0)
        short = minehip.multi_plan(b"cmu440", 0, hi - n, n)
        assert [s["kind"] for s in short] == [0] * n
    # configs[4] (2^42) over 8 GPU miners: heads of ~5e11 nonces and 16 tail chunks of ~1.7e10
    spans = minehip.multi_plan(b"cmu440", 0, (1 << 42) - 1, 8)
    assert sum(s["kind"] for s in spans) == 16
    assert len(minehip.multi_plan(b"cmu440", 0, (1 << 42) - 1, 1)) == 1  # one worker: no tail


def test_split_argument_errors():
    with pytest.raises(minehip.MinehipError) as e:
        minehip.multi_plan(b"x", 5, 4, 2)
    assert e.value.code == minehip.MH_ERANGE
    with pytest.raises(minehip.MinehipError) as e:
        minehip.multi_plan(b"x", 0, 4, 2, [1.0, 0.0])
    assert e.value.code == minehip.MH_EINVAL
    for bad in (float("inf"), float("nan"), -1.0):
        with pytest.raises(minehip.MinehipError):
            minehip.multi_plan(b"x", 0, 4, 2, [1.0, bad])
    with pytest.raises(minehip.MinehipError) as e:
        minehip.multi_plan(b"x", 0, 4, 0)
    assert e.value.code == minehip.MH_EINVAL
    with pytest.raises(minehip.MinehipError) as e:  # one host thread per listed device: bounded
        minehip.multi_plan(b"x", 0, 4, minehip._lib.MH_MAX_WORKERS + 1)
    assert e.value.code == minehip.MH_EINVAL
    assert len(minehip.multi_plan(b"x", 0, 10 ** 6, minehip._lib.MH_MAX_WORKERS)) == minehip._lib.MH_MAX_WORKERS
    # a weight per worker, no more and no fewer (a short list was zero-padded by ctypes)
    for w in ([1.0], [1.0, 1.0, 1.0]):
        with pytest.raises(ValueError):
            minehip.multi_plan(b"x", 0, 4, 2, w)


def test_rate_table_starts_empty():
    assert minehip.multi_rates([0, 1, 7]) == [0.0, 0.0, 0.0]
    # an empty device list is no error, whatever the pointers
    assert minehip.lib.mh_multi_rates(None, 0, None) == 0
    assert minehip.multi_rates([]) == []
