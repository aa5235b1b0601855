"""CPU checks of the full-size fixtures (tests/golden/fullsize_<cfg>.json) that
tests/test_gpu_fullsize.py and bench.py hold the HIP path to.

The fixtures were scanned with OpenSSL's SHA-256 (tests/golden/gen_fullsize.py);
here they must be self-consistent and agree with the C oracle restatement of
bitcoin/hash.go:13-17 + the A2 scan spec on sampled chunks.
"""
import os

import pytest

from conftest import load_golden
from oracle import oracle

CFGS = {"cfg2": (b"cmu440", (1 << 35) - 1), "cfg3a": (b"a" * 100, (1 << 34) - 1),
        "cfg3b": (b"x" * 60, (1 << 34) - 1)}


@pytest.mark.parametrize("name", sorted(CFGS))
def test_fixture_consistent(name):
    d = load_golden(f"fullsize_{name}.json")
    msg, hi = CFGS[name]
    assert bytes.fromhex(d["msg_hex"]) == msg and d["lo"] == 0 and d["hi"] == hi
    chunks = [tuple(c) for c in d["chunks"]]
    size = 1 << d["chunk_bits"]
    assert len(chunks) == (hi + 1) // size
    assert tuple(d["result"]) == min(chunks)
    for i, (h, n) in enumerate(chunks):
        assert i * size <= n < (i + 1) * size
        if i % 97 == 0:
            assert oracle.hash_(msg, n) == h


@pytest.mark.parametrize("name", sorted(CFGS))
def test_fixture_chunk_vs_oracle(name):
    d = load_golden(f"fullsize_{name}.json")
    msg, _ = CFGS[name]
    size = 1 << d["chunk_bits"]
    i = {"cfg2": 255, "cfg3a": 611, "cfg3b": 1000}[name]  # d = 10, 11, 11 chunks
    got = oracle.search(msg, i * size, (i + 1) * size - 1, threads=os.cpu_count() or 1)
    assert got == tuple(d["chunks"][i])


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
