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
  cfg4s  "cmu440": 100 chunks sampled from configs[3]/[4] ([0, 2^42-1], d = 11..13)

Reference semantics: bitcoin/hash.go:13-17 and the scan spec of SURVEY.md
§8(a) A2 (reference stub bitcoin/miner/miner.go:33).
"""
import pytest

from conftest import load_golden
from test_gpu_parity import env

pytestmark = pytest.mark.gpu

CFGS = ("cfg2", "cfg3a", "cfg3b")


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


def test_plan_knobs_full_size(gpu):
    """The answer at 2^32 does not depend on the launch plan."""
    msg, _, _, bits, _, chunks = fixture("cfg2")
    exp = min(chunks[:(1 << 32) >> bits])
    for kv in (dict(MINEHIP_LOWER_DIGITS=1), dict(MINEHIP_LOWER_DIGITS=3, MINEHIP_MIN_LANES=1 << 18),
               dict(MINEHIP_LAUNCH_NONCES=1 << 28), dict(MINEHIP_GENERIC_BELOW=0)):
        with env(**kv):
            assert gpu.search(msg, 0, (1 << 32) - 1) == exp, kv


def test_search_multi_full_size(gpu):
    """The scheduler path (one miner per device, chunked) at 2^34 with two tail blocks."""
    msg, lo, hi, _, result, _ = fixture("cfg3b")
    assert gpu.search_multi(msg, lo, hi, devs=[0]) == result
