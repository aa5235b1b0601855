"""GPU parity at BASELINE.json's full sizes, bit-exact against fixtures.

tests/golden/fullsize_<cfg>.json hold the (hash, nonce) minimum of every
2^24-nonce chunk and of the whole range, scanned once with OpenSSL's SHA-256
(tests/golden/gen_fullsize.py; cross-checked there against oracle/ and
hashlib).  Here the HIP path (C-ABI mh_search / mh_search_multi) must
reproduce every one of them:

  cfg2   "cmu440" [0, 2^35-1]: configs[1] ([0, 2^32-1], every digit bucket
         d = 1..10) and the union of bench.py's weak-scaling shards at 8 GPUs
  cfg3a  "a" x 100 [0, 2^34-1]: configs[2], host-midstate block
  cfg3b  "x" x 60  [0, 2^34-1]: configs[2], two tail blocks
  two13, two14, two15, pre0, pre2
         ("cmu440-" repeated)[:n], n = 45/48/52/55/62, [0, 2^32-1]: the d = 10
         bucket in the two-block layouts fast_search<13..15, Two> and
         fast_search<0, Pre>, <2, Pre> (cfg3b is <1, Pre>), lower buckets in others
  one1, one5, one7, one8, one10, one12
         ("cmu440-" repeated)[:n], n = 0/13/21/25/30/41, [0, 2^32-1]: one tail block,
         d = 7..10 in <1|2|5|7|8|9|10|12, One>; with the rest every layout the
         default plan uses (test_fullsize_fixtures.py checks the coverage).  Where a
         bucket's default layout is an Early one (<0|8, OneEarly>, <0, PreEarly>,
         <13, TwoEarly>: cfg3b, two14, two15, pre2, one1, one10) the named last-digit
         kernel runs with MINEHIP_EARLY=0, and both are checked
  pre3, pre4, top
         2^32 nonces from 10^13 and 10^17 for the 62-byte message (<3, Pre>, <4, Pre>),
         and "cmu440" over [2^64-2^32, 2^64-1] (20 digits, <6, One>, up to the last u64)
  cfg4s  "cmu440": 100 chunks sampled from configs[3]/[4] ([0, 2^42-1], d = 11..13)
  cfg4   "cmu440" [0, 2^40-1]: configs[3] whole, its 256 2^32-chunk minima
         (tests/golden/gen_cfg4.py: SHA-NI scan, checked against OpenSSL)
  cfg5s  "cmu440": 64 sampled 2^28 chunks of [2^40, 2^42-1] (tests/golden/gen_cfg5s.py, SHA-NI)
  cfg5c  "cmu440" [1017 * 2^32, 1018 * 2^32 - 1]: the 2^32 chunk of configs[4] that holds its
         answer, in 2^28 chunks (tests/golden/gen_cfg5c.py: SHA-NI scan, checked against OpenSSL);
         configs[4] itself runs in test_e2e_cluster.py (direct and over LSP with 8 miners)

Reference semantics: bitcoin/hash.go:13-17 and the scan spec of SURVEY.md
§8(a) A2 (reference stub bitcoin/miner/miner.go:33).
"""
import os

import pytest

from conftest import GOLDEN, load_golden
from test_gpu_parity import env

pytestmark = pytest.mark.gpu

CFGS = ("cfg2", "cfg3a", "cfg3b", "two13", "two14", "two15", "pre0", "pre2", "pre3", "pre4", "top",
        "one1", "one5", "one7", "one8", "one10", "one12", "cfg5c")


def fixture(name):
    d = load_golden(f"fullsize_{name}.json")
    return (bytes.fromhex(d["msg_hex"]), int(d["lo"]), int(d["hi"]), int(d["chunk_bits"]),
            tuple(d["result"]), [tuple(c) for c in d["chunks"]])


@pytest.mark.parametrize("name", CFGS)
def test_every_chunk(gpu, name):
    msg, lo, hi, bits, _, chunks = fixture(name)
    size = 1 << bits
    bad = []
    for i, exp in enumerate(chunks):
        a = lo + i * size
        got = gpu.search(msg, a, min(hi, a + size - 1))
        if got != exp:
            bad.append((i, got, exp))
    assert not bad, f"{len(bad)} of {len(chunks)} chunks differ, first: {bad[:3]}"


@pytest.mark.parametrize("name", CFGS)
def test_whole_range(gpu, name):
    msg, lo, hi, _, result, _ = fixture(name)
    assert gpu.search(msg, lo, hi) == result


# the fixtures whose default plan takes an Early layout (the digit ending the word before the last
# digit's innermost, fast_search<J, 3..5>): the same chunks and whole range with MINEHIP_EARLY=0,
# on the last-digit kernels the Early ones replace, so both orders are pinned at full size
EARLY = ("cfg3b", "two14", "two15", "pre2", "one1", "one10")


@pytest.mark.parametrize("name", EARLY)
def test_every_chunk_last_digit_innermost(gpu, name):
    msg, lo, hi, bits, result, chunks = fixture(name)
    size = 1 << bits
    with env(MINEHIP_EARLY=0):
        bad = [(i, exp) for i, exp in enumerate(chunks)
               if gpu.search(msg, lo + i * size, min(hi, lo + (i + 1) * size - 1)) != exp]
        assert not bad, f"{len(bad)} of {len(chunks)} chunks differ, first: {bad[:3]}"
        assert gpu.search(msg, lo, hi) == result


def test_config2_and_shards(gpu):
    """configs[1] exactly, and each weak-scaling shard [r*2^32, (r+1)*2^32-1] of bench.py."""
    msg, lo, hi, bits, _, chunks = fixture("cfg2")
    per = (1 << 32) >> bits
    for r in range(8):
        exp = min(chunks[r * per:(r + 1) * per])
        assert gpu.search(msg, r << 32, ((r + 1) << 32) - 1) == exp, r
    assert gpu.search(msg, 0, (1 << 32) - 1) == min(chunks[:per])


def test_config4_5_samples(gpu):
    """configs[3]/[4] ranges ([0, 2^40-1], [0, 2^42-1]; d = 11..13): 100 OpenSSL-scanned 2^24 chunks."""
    d = load_golden("fullsize_cfg4s.json")
    msg = bytes.fromhex(d["msg_hex"])
    bad = [(lo, hi) for lo, hi, h, n in d["samples"] if gpu.search(msg, lo, hi) != (h, n)]
    assert not bad, bad[:3]


def test_config5_sampled_chunks(gpu):
    """BASELINE configs[4] ([0, 2^42-1]) above configs[3]: [2^40, 2^42) is pinned on the CPU by 64
    sampled 2^28-nonce chunks (tests/golden/gen_cfg5s.py: SHA-NI, one chunk rescanned with OpenSSL;
    VERDICT r05 item 3).  Every chunk searched on the GPU gives its CPU minimum, and the answer
    chunk's minimum (fullsize_cfg5c.json: configs[4]'s answer) beats every sample."""
    d = load_golden("fullsize_cfg5s.json")
    msg = bytes.fromhex(d["msg_hex"])
    assert (d["lo"], d["hi"]) == (1 << 40, (1 << 42) - 1) and len(d["samples"]) >= 64
    bad = [(lo, hi) for lo, hi, h, n in d["samples"] if gpu.search(msg, lo, hi) != (h, n)]
    assert not bad, bad[:3]
    answer = tuple(load_golden("fullsize_cfg5c.json")["result"])
    assert all(answer < (h, n) for _, _, h, n in d["samples"])


def test_plan_knobs_full_size(gpu):
    """The answer at 2^32 does not depend on the launch plan."""
    msg, _, _, bits, _, chunks = fixture("cfg2")
    exp = min(chunks[:(1 << 32) >> bits])
    for kv in (dict(MINEHIP_LOWER_DIGITS=1), dict(MINEHIP_LOWER_DIGITS=3, MINEHIP_MIN_LANES=1 << 18),
               dict(MINEHIP_LAUNCH_NONCES=1 << 28), dict(MINEHIP_GENERIC_BELOW=0),
               dict(MINEHIP_STREAMS=2), dict(MINEHIP_STREAMS=2, MINEHIP_LAUNCH_NONCES=1 << 30,
                                             MINEHIP_MAX_BLOCKS=1 << 12),
               dict(MINEHIP_STREAMS=2, MINEHIP_FINE_TAIL=1 << 28), dict(MINEHIP_FINE_TAIL=(1 << 30) + 12345)):
        with env(**kv):
            assert gpu.search(msg, 0, (1 << 32) - 1) == exp, kv


@pytest.mark.parametrize("name", ("two15", "pre0"))
def test_plan_knobs_two_block_layouts(gpu, name):
    """The two-block layouts at 2^32 under other lane run lengths, launch sizes and with every
    bucket on the fast kernels: the answer stays the fixture's."""
    msg, lo, hi, _, result, _ = fixture(name)
    for kv in (dict(MINEHIP_LOWER_DIGITS=1), dict(MINEHIP_LOWER_DIGITS=3, MINEHIP_MIN_LANES=1 << 18),
               dict(MINEHIP_LAUNCH_NONCES=1 << 28), dict(MINEHIP_GENERIC_BELOW=0),
               dict(MINEHIP_STREAMS=2, MINEHIP_FINE_TAIL=1 << 28, MINEHIP_MIN_LANES=1 << 18)):
        with env(**kv):
            assert gpu.search(msg, lo, hi) == result, kv


def test_search_multi_full_size(gpu):
    """The scheduler path (one miner per device, chunked) at 2^34 with two tail blocks; one
    listed device takes the direct path (a single search), two take the scheduler."""
    msg, lo, hi, _, result, _ = fixture("cfg3b")
    assert gpu.search_multi(msg, lo, hi, devs=[0]) == result
    assert gpu.search_multi(msg, lo, hi, devs=[0, 0]) == result


CFG4_HI = (1 << 40) - 1


def _cfg4_checks(gpu, got):
    """configs[3]'s answer, checked by everything that pins it without a second 2^40 scan."""
    msg = b"cmu440"
    assert gpu.Hash(msg, got[1]) == got[0]                # re-hashed by the generic kernel
    assert 0 <= got[1] <= CFG4_HI
    whole35 = fixture("cfg2")[4]                          # [0, 2^35-1] is a prefix of the range
    assert got <= whole35 and (got[1] >= 1 << 35 or got == whole35)
    d = load_golden("fullsize_cfg4s.json")
    below = [(h, n) for lo, hi, h, n in d["samples"] if hi <= CFG4_HI]
    assert below and all(got <= s for s in below)         # no sampled chunk beats it
    path = os.path.join(GOLDEN, "fullsize_cfg4.json")
    if os.path.exists(path):                              # the full CPU scan of [0, 2^40-1]
        f = load_golden("fullsize_cfg4.json")
        assert (f["lo"], f["hi"]) == (0, CFG4_HI)
        assert got == tuple(f["result"])


def test_config3_full_range(gpu):
    """BASELINE configs[3] at its stated size on one GPU: "cmu440" over [0, 2^40-1] (~33 s)."""
    _cfg4_checks(gpu, gpu.search(b"cmu440", 0, CFG4_HI))


def test_config3_full_range_multi(gpu):
    """The same 2^40 range through mh_search_multi with eight worker threads (one host thread +
    stream each, all on device 0): the scheduler's chunking, fair-share tail and host merge."""
    _cfg4_checks(gpu, gpu.search_multi(b"cmu440", 0, CFG4_HI, devs=[0] * 8))


def test_config3_chunks_against_fixture(gpu):
    """Eight of configs[3]'s 2^32-nonce chunk minima (first, last, the 10^11 and 10^12 buckets)."""
    path = os.path.join(GOLDEN, "fullsize_cfg4.json")
    if not os.path.exists(path):
        pytest.skip("tests/golden/fullsize_cfg4.json not generated")
    f = load_golden("fullsize_cfg4.json")
    size = 1 << f["chunk_bits"]
    picks = sorted({0, 8, 23, 24, 232, 233, 254, 255})
    for i in picks:
        a = f["lo"] + i * size
        assert gpu.search(b"cmu440", a, a + size - 1) == tuple(f["chunks"][i]), i
