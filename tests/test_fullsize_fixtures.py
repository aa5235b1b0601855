"""CPU checks of the full-size fixtures (tests/golden/fullsize_<cfg>.json) that
tests/test_gpu_fullsize.py and bench.py hold the HIP path to.

The fixtures were scanned with OpenSSL's SHA-256 (tests/golden/gen_fullsize.py);
here they must be self-consistent and agree with the C oracle restatement of
bitcoin/hash.go:13-17 + the A2 scan spec on sampled chunks.
"""
import os

import pytest

from conftest import GOLDEN, load_golden
from oracle import oracle

CFGS = {"cfg2": (b"cmu440", (1 << 35) - 1), "cfg3a": (b"a" * 100, (1 << 34) - 1),
        "cfg3b": (b"x" * 60, (1 << 34) - 1)}
# tail layouts of the d = 10 bucket that BASELINE's messages do not reach (gen_fullsize.py)
LAYOUTS = {"two13": 45, "two14": 48, "two15": 52, "pre0": 55, "pre2": 62,
           "one1": 0, "one5": 13, "one7": 21, "one8": 25, "one10": 30, "one12": 41}
CFGS.update({k: ((b"cmu440-" * 10)[:n], (1 << 32) - 1) for k, n in LAYOUTS.items()})
# (msg, hi, lo) for the ranges that do not start at 0: the 14-/18-digit buckets and the top of u64
CFGS.update({"pre3": ((b"cmu440-" * 10)[:62], 10 ** 13 + (1 << 32) - 1, 10 ** 13),
             "pre4": ((b"cmu440-" * 10)[:62], 10 ** 17 + (1 << 32) - 1, 10 ** 17),
             "top": (b"cmu440", (1 << 64) - 1, (1 << 64) - (1 << 32))})
# BASELINE configs[4]'s answer chunk, [1017 * 2^32, 1018 * 2^32 - 1] in 2^28 chunks (gen_cfg5c.py, SHA-NI)
CFGS["cfg5c"] = (b"cmu440", (1018 << 32) - 1, 1017 << 32)


def _cfg(name):
    msg, hi, *lo = CFGS[name]
    return msg, (lo[0] if lo else 0), hi


@pytest.mark.parametrize("name", sorted(CFGS))
def test_fixture_consistent(name):
    d = load_golden(f"fullsize_{name}.json")
    msg, lo, hi = _cfg(name)
    assert bytes.fromhex(d["msg_hex"]) == msg and d["lo"] == lo and d["hi"] == hi
    chunks = [tuple(c) for c in d["chunks"]]
    size = 1 << d["chunk_bits"]
    assert len(chunks) == (hi - lo + 1) // size
    assert tuple(d["result"]) == min(chunks)
    for i, (h, n) in enumerate(chunks):
        assert lo + i * size <= n < lo + (i + 1) * size
        if i % 97 == 0:
            assert oracle.hash_(msg, n) == h


@pytest.mark.parametrize("name", sorted(CFGS))
def test_fixture_chunk_vs_oracle(name):
    d = load_golden(f"fullsize_{name}.json")
    msg, lo, _ = _cfg(name)
    size = 1 << d["chunk_bits"]
    i = {"cfg2": 255, "cfg3a": 611, "cfg3b": 1000, "cfg5c": 15}.get(name, 255)  # cfg*: d = 10, 11, 11; the rest: last
    got = oracle.search(msg, lo + i * size, lo + (i + 1) * size - 1, threads=os.cpu_count() or 1)
    assert got == tuple(d["chunks"][i])


def test_config5_sample_fixture():
    """fullsize_cfg5s.json: 64 2^28-nonce chunks spread over [2^40, 2^42), the
    range's first and last chunk among them, as gen_cfg5s.sample_los() draws them; every minimum
    re-hashes through the oracle and lies in its chunk; one chunk is rescanned by the oracle; the
    answer chunk's minimum (configs[4]'s answer, fullsize_cfg5c.json) beats every sample."""
    import sys
    sys.path.insert(0, GOLDEN)
    import gen_cfg5s
    d = load_golden("fullsize_cfg5s.json")
    assert bytes.fromhex(d["msg_hex"]) == b"cmu440" and (d["lo"], d["hi"]) == (1 << 40, (1 << 42) - 1)
    los = [s[0] for s in d["samples"]]
    assert los == gen_cfg5s.sample_los() and len(los) == 64
    assert los[0] == 1 << 40 and d["samples"][-1][1] == (1 << 42) - 1
    stride = 3 << 34
    assert all((los[i] - (1 << 40)) // stride == i for i in range(64))  # one per 3 * 2^34 stride
    for lo, hi, h, n in d["samples"]:
        assert hi - lo + 1 == 1 << d["chunk_bits"] == 1 << 28 and lo <= n <= hi
        assert oracle.hash_(b"cmu440", n) == h
    lo, hi, h, n = d["samples"][0]
    assert oracle.search(b"cmu440", lo, hi, threads=os.cpu_count() or 1) == (h, n)
    answer = tuple(load_golden("fullsize_cfg5c.json")["result"])
    assert all(answer < (h, n) for _, _, h, n in d["samples"])


def test_sample_fixture():
    d = load_golden("fullsize_cfg4s.json")
    assert bytes.fromhex(d["msg_hex"]) == b"cmu440" and len(d["samples"]) == 100
    los = [s[0] for s in d["samples"]]
    assert los == sorted(set(los))
    for lo, hi, h, n in d["samples"]:
        assert hi - lo + 1 == 1 << d["chunk_bits"] and lo <= n <= hi and hi < 1 << 42
    for lo, hi, h, n in d["samples"][::33]:
        assert oracle.hash_(b"cmu440", n) == h
    lo, hi, h, n = d["samples"][50]
    assert oracle.search(b"cmu440", lo, hi, threads=os.cpu_count() or 1) == (h, n)


def test_config3_fixture():
    """fullsize_cfg4.json (configs[3] whole, [0, 2^40-1] in 2^32 chunks; gen_cfg4.py): tiles the
    range, agrees with fullsize_cfg2.json on [0, 2^35) and with every OpenSSL-scanned sample chunk
    of fullsize_cfg4s.json below 2^40, and re-hashes through the oracle."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize_cfg4.json")
    if not os.path.exists(path):
        pytest.skip("tests/golden/fullsize_cfg4.json not generated")
    d = load_golden("fullsize_cfg4.json")
    assert bytes.fromhex(d["msg_hex"]) == b"cmu440" and d["lo"] == 0 and d["hi"] == (1 << 40) - 1
    size = 1 << d["chunk_bits"]
    chunks = [tuple(c) for c in d["chunks"]]
    assert len(chunks) == (1 << 40) // size and tuple(d["result"]) == min(chunks)
    for i, (h, n) in enumerate(chunks):
        assert i * size <= n < (i + 1) * size
        if i % 17 == 0:
            assert oracle.hash_(b"cmu440", n) == h
    d2 = load_golden("fullsize_cfg2.json")
    per = size >> d2["chunk_bits"]
    for i in range((1 << 35) // size):
        assert chunks[i] == min(tuple(c) for c in d2["chunks"][i * per:(i + 1) * per])
    for lo, hi, h, n in load_golden("fullsize_cfg4s.json")["samples"]:
        if hi < 1 << 40:
            c = chunks[lo // size]
            assert lo // size == hi // size and c <= (h, n)
            if lo <= c[1] <= hi:
                assert c == (h, n)


# the last-digit layouts an Early layout replaces in the default plan of every bucket holding two
# blocks of its lanes (10^(p+L) nonces each, up to 10^7); MINEHIP_EARLY=0 plans them instead
REPLACED_BY_EARLY = {(1, 0), (1, 1), (9, 0), (14, 2)}
EARLY_FIXTURES = ("cfg3b", "two14", "two15", "pre2", "one1", "one10")


def _used(names, early):
    import minehip
    old = os.environ.get("MINEHIP_EARLY")
    os.environ["MINEHIP_EARLY"] = str(early)
    try:
        used = set()
        for name in names:
            msg, lo, hi = _cfg(name)
            used |= {(p["word"], p["mode"]) for p in minehip.plan(msg, lo, hi) if p["kind"] == 0}
        if early:
            for lo, hi, _, _ in load_golden("fullsize_cfg4s.json")["samples"]:
                used |= {(p["word"], p["mode"]) for p in minehip.plan(b"cmu440", lo, hi) if p["kind"] == 0}
        return used
    finally:
        if old is None:
            os.environ.pop("MINEHIP_EARLY")
        else:
            os.environ["MINEHIP_EARLY"] = old


def test_fixtures_cover_every_fast_layout():
    """The default plans of the full-size fixtures' ranges (host-only mh_plan) use every
    fast_search<J, MODE> instantiation the default plan chooses for a bucket of more than two
    Early blocks: all 26 but <0, One>, whose last digit would sit in message bytes 0..3, i.e.
    d <= 4 -- always a bucket of fewer than 2^20 nonces, which goes to the generic kernel --
    and the four last-digit layouts the Early ones replace.  Those four are what
    the same fixtures plan with MINEHIP_EARLY=0 (tests/test_gpu_fullsize.py runs both)."""
    from test_abi import KERNELS
    used = _used(CFGS, 1)
    # (the replaced kernels may still run an Early bucket's ragged ends, in runs of 10^L)
    assert KERNELS - {(0, 0)} - REPLACED_BY_EARLY <= used <= KERNELS - {(0, 0)}, sorted(KERNELS - used)
    assert _used(EARLY_FIXTURES, 0) >= REPLACED_BY_EARLY
    for name in EARLY_FIXTURES:  # exactly these fixtures change kernels with the knob
        assert _used((name,), 1) != _used((name,), 0), name
