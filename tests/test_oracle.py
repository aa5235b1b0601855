"""Pins the CPU oracle (oracle/sha256_oracle.c) before anything trusts it.

- FIPS 180-4 published known answers (the standard Go's crypto/sha256 -- the
  reference's arithmetic, bitcoin/hash.go:6,14 -- implements),
- the hashlib-generated golden fixtures of tests/golden/ (gen_golden.py),
- the survey's known answers.
"""
import hashlib
import random

import numpy as np
import pytest

from conftest import load_golden
from oracle import oracle


def test_fips180_4_vectors():
    d = load_golden("fips180_4.json")
    for v in d["vectors"]:
        assert oracle.sha256(bytes.fromhex(v["msg_hex"])).hex() == v["sha256"]
    assert oracle.sha256(b"a" * 1000000).hex() == d["million_a"]


def test_sha256_against_hashlib_every_length():
    rng = random.Random(7)
    for n in list(range(0, 200)) + [447, 448, 511, 512, 513, 1000, 4096]:
        m = bytes(rng.getrandbits(8) for _ in range(n))
        assert oracle.sha256(m) == hashlib.sha256(m).digest(), n


def test_hash_golden_vectors(golden_hash):
    by_msg = {}
    for m, n, h in golden_hash:
        by_msg.setdefault(m, []).append((n, h))
    for m, lst in by_msg.items():
        nonces = np.array([n for n, _ in lst], dtype=np.uint64)
        got = oracle.hash_batch(m, nonces)
        exp = np.array([h for _, h in lst], dtype=np.uint64)
        assert (got == exp).all(), m[:20]


def test_survey_known_answers():
    assert oracle.hash_("cmu440", 0) == 11864962392530079502
    assert oracle.hash_("cmu440", 1) == 6607435123466727425
    assert oracle.hash_("cmu440", 9999999) == 3708070381600383132
    assert oracle.hash_("cmu440", 4294967295) == 18396963905960875035
    assert oracle.hash_("cmu440", 18446744073709551615) == 12656178859598403723
    assert oracle.hash_("", 0) == 17297653956949303043


def test_scan_golden(golden_scan):
    small, _ = golden_scan
    for m, lo, hi, h, n in small:
        assert oracle.search(m, lo, hi) == (h, n), (m[:16], lo, hi)
        assert oracle.search(m, lo, hi, threads=3) == (h, n)


def test_scan_config1(golden_scan):
    _, big = golden_scan
    m, lo, hi, h, n = big[0]
    assert (h, n) == (1228377698034, 1067492)
    assert oracle.search(m, lo, hi, threads=8) == (h, n)


def test_scan_edges():
    U = (1 << 64) - 1
    assert oracle.search("cmu440", U, U) == (oracle.hash_("cmu440", U), U)
    with pytest.raises(ValueError):
        oracle.search("cmu440", 5, 4)
    # strict-< first minimum == lexicographic (hash, nonce) minimum
    lo, hi = 1000, 3000
    hs = oracle.hash_batch("tie", np.arange(lo, hi + 1, dtype=np.uint64))
    k = int(np.argmin(hs))
    assert oracle.search("tie", lo, hi) == (int(hs[k]), lo + k)


def test_openssl_scan_matches_restatement():
    """oracle/openssl_scan.c (bench.py's tuned CPU baseline) answers like the restatement."""
    U = (1 << 64) - 1
    cases = [(b"cmu440", 0, 99_999), (b"cmu440", 9_990, 10_010), (b"", 0, 5_000), (b"x" * 60, 95_000, 105_000),
             (b"a" * 100, 7, 7), (b"cmu440", U - 3_000, U), (bytes(range(256)), 10 ** 12 - 500, 10 ** 12 + 500)]
    for msg, lo, hi in cases:
        for threads in (1, 3):
            assert oracle.search_openssl(msg, lo, hi, threads=threads) == oracle.search(msg, lo, hi), (msg[:8], lo, hi)
    with pytest.raises(ValueError):
        oracle.search_openssl(b"m", 5, 4)
