"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle and the
golden fixtures.  Bit-exact (integer work).  Reference semantics:
bitcoin/hash.go:13-17 (Hash) and the miner scan spec (SURVEY.md §8(a) A2,
reference stub bitcoin/miner/miner.go:33).

Small sizes are checked element for element against oracle/; BASELINE.json's
full sizes (2^32 and 2^34 nonces) are checked through size-independent
properties: split-range associativity of the min, invariance to the launch
plan (lower-digit count L, launch size, device chunking), and that the
reported (hash, nonce) re-hashes to itself.
"""
import os
import random

import numpy as np
import pytest

from oracle import oracle
from conftest import ROOT

pytestmark = pytest.mark.gpu

U64 = (1 << 64) - 1


def lexmin(a, b):
    return a if a <= b else b


class env:
    """Temporarily set planner knobs (read by libminehip on every search)."""

    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def both_paths():
    """Small ranges run once on the fast kernels (MINEHIP_GENERIC_BELOW=0) and
    once as the default plan, which sends buckets < 2^20 nonces to the
    generic kernel."""
    return (env(MINEHIP_GENERIC_BELOW=0), env())


def test_hash_batch_golden(gpu, golden_hash):
    by_msg = {}
    for m, n, h in golden_hash:
        by_msg.setdefault(m, []).append((n, h))
    for m, lst in by_msg.items():
        got = gpu.hash_batch(m, np.array([n for n, _ in lst], dtype=np.uint64))
        exp = np.array([h for _, h in lst], dtype=np.uint64)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (m[:20], [lst[i] for i in bad[:3]])


def test_hash_single(gpu):
    assert gpu.Hash("cmu440", 0) == 11864962392530079502
    assert gpu.Hash("cmu440", U64) == 12656178859598403723
    assert gpu.Hash("", 0) == 17297653956949303043


def test_hash_batch_random_vs_oracle(gpu):
    rng = np.random.default_rng(440)
    for L in (0, 1, 7, 54, 55, 56, 62, 63, 64, 118, 119, 200, 601):
        m = bytes(rng.integers(32, 127, size=L, dtype=np.uint8))
        nonces = rng.integers(0, U64, size=5000, dtype=np.uint64, endpoint=True)
        nonces[:20] = [10 ** k for k in range(20)]
        assert (gpu.hash_batch(m, nonces) == oracle.hash_batch(m, nonces)).all(), L
    assert gpu.hash_batch("x", []).size == 0


def test_scan_golden(gpu, golden_scan):
    small, big = golden_scan
    for m, lo, hi, h, n in small:
        assert gpu.search(m, lo, hi) == (h, n), (m[:16], lo, hi)


def test_config1(gpu, golden_scan):
    """BASELINE.json configs[0]: "cmu440", nonces 0..9,999,999."""
    _, big = golden_scan
    m, lo, hi, h, n = big[0]
    assert gpu.search(m, lo, hi) == (h, n) == (1228377698034, 1067492)


def test_every_tail_offset_and_bucket(gpu):
    """Every prefix length mod 64 (all fast-kernel layouts J / modes) and
    ranges straddling 10^k for many k, against the oracle."""
    rng = random.Random(440)
    for L in range(0, 131):
        m = bytes(rng.choice(b"abcdefghij ") for _ in range(L))
        for k in rng.sample(range(2, 20), 3) + [19]:
            c = 10 ** k
            lo = max(0, c - rng.randrange(1000, 9000))
            hi = min(U64, c + rng.randrange(3000, 14000))
            exp = oracle.search(m, lo, hi, threads=8)
            for e in both_paths():
                with e:
                    assert gpu.search(m, lo, hi) == exp, (L, lo, hi, e.kv)


def test_every_kernel_instantiation(gpu):
    """Each of the 26 fast_search<J, MODE> kernels, at the shortest and the
    longest lane runs (L = 1 and the largest L the layout allows), bit-exact
    against the oracle over ranges holding whole runs (an Early layout: whole
    blocks of interleaved lanes) plus ragged edges."""
    from test_abi import KERNELS, KERNEL_CASE_NONCES, kernel_cases
    cases = kernel_cases()
    assert set(cases) == KERNELS
    for (J, mode), (m, lo, _, early) in sorted(cases.items()):
        hi = lo + KERNEL_CASE_NONCES + 3_456
        exp = oracle.search(m, lo, hi, threads=8)
        for Ld in (1, 3):
            with env(MINEHIP_LOWER_DIGITS=Ld, MINEHIP_MIN_LANES=1, MINEHIP_GENERIC_BELOW=0, MINEHIP_EARLY=early):
                assert gpu.search(m, lo, hi) == exp, (J, mode, len(m), Ld)


def early_position_cases(Ls=(1, 2, 3), max_p=4):
    """(msg, lo, hi, L, J, mode, p) for every (Early kernel, innermost position p, L) the planner
    can produce: messages of every tail offset, each bucket d = 2..20 from its first nonce (and
    the top of the u64 range for d = 20), two blocks of lanes (10^(p+L) nonces each, p <= max_p)
    plus a ragged edge.  Host only."""
    import minehip
    cases = {}
    for n in range(0, 128):
        m = b"q" * n
        t = (n + 1) % 64
        for d in range(2, 21):
            for Ld in Ls:
                with env(MINEHIP_LOWER_DIGITS=Ld, MINEHIP_MIN_LANES=1, MINEHIP_GENERIC_BELOW=0):
                    size = 2 * 10 ** (max_p + Ld) + 3_456  # two blocks at p = max_p
                    los = [10 ** (d - 1)] + ([U64 - size] if d == 20 else [])
                    for lo in los:
                        hi = min(U64, lo + size)
                        for pc in minehip.plan(m, lo, hi):
                            if pc["kind"] != 0 or pc["mode"] < 3:
                                continue
                            pl = t + pc["digits"] - 1
                            base = 64 if (pc["blocks"] == 2 and pl >= 64) else 0
                            pos = pl - (base + 4 * pc["word"] + 3)
                            assert 1 <= pos <= 4 and pc["first"] % 10 ** (pos + pc["lo_digits"]) == 0, (n, lo, pc)
                            key = (pc["word"], pc["mode"], pos, pc["lo_digits"], lo == los[-1] and d == 20)
                            cases.setdefault(key, (m, lo, hi, Ld))
    return cases


def test_early_layout_every_position(gpu):
    """Each Early kernel (the digit ending word J innermost) at every decimal position p of that
    digit and every lane length L it is planned with -- contiguous lanes (p < L, the group digits
    around p) and interleaved ones (p >= L, U's digits around p) -- and at the top of the u64
    range: bit-exact against the oracle, and against the last-digit plan (MINEHIP_EARLY=0)."""
    cases = early_position_cases()
    kinds = {(J, mode) for (J, mode, *_rest) in cases}
    assert kinds == {(0, 3), (8, 3), (0, 4), (13, 5)}, kinds
    assert any(p < L for (_, _, p, L, _) in cases) and any(p >= L for (_, _, p, L, _) in cases)
    # L = 4 (MINEHIP_LOWER_DIGITS >= 4): the whole of word J enumerated, the group three digits;
    # at p = 1 (two blocks are 2 x 10^5 nonces, oracle-sized), one case per Early kernel that
    # plans at L = 4.  <0, OneEarly> never does: word 0 all digits puts the first
    # digit at byte 0, so p = d - 4 and a block of 10^(p+4) = 10^d nonces exceeds its bucket
    cases4 = early_position_cases(Ls=(4,), max_p=1)
    assert {(J, mode) for (J, mode, *_rest) in cases4} == kinds - {(0, 3)}, cases4.keys()
    assert all(p == 1 and L == 4 for (_, _, p, L, _) in cases4)
    for key, (m, lo, hi, Ld) in sorted(cases.items()) + sorted(cases4.items()):
        exp = oracle.search(m, lo, hi, threads=8)
        with env(MINEHIP_LOWER_DIGITS=Ld, MINEHIP_MIN_LANES=1, MINEHIP_GENERIC_BELOW=0):
            assert gpu.search(m, lo, hi) == exp, (key, len(m), lo, hi)
            with env(MINEHIP_EARLY=0):
                assert gpu.search(m, lo, hi) == exp, (key, "last digit")


def test_u64_edges(gpu):
    for m in (b"cmu440", b"", b"q" * 60, b"r" * 119):
        top = oracle.search(m, U64 - 30000, U64, threads=8)
        low = oracle.search(m, 0, 25000, threads=8)
        for e in both_paths():
            with e:
                assert gpu.search(m, U64, U64) == (oracle.hash_(m, U64), U64)
                assert gpu.search(m, U64 - 30000, U64) == top
                assert gpu.search(m, 0, 0) == (oracle.hash_(m, 0), 0)
                assert gpu.search(m, 0, 25000) == low


def test_long_messages(gpu):
    for L in (191, 192, 300, 447, 600, 1000, 5000):
        m = bytes((i * 7 + 3) % 95 + 32 for i in range(L))
        exp = oracle.search(m, 999000, 1012000, threads=8)
        for e in both_paths():
            with e:
                assert gpu.search(m, 999000, 1012000) == exp, L


def test_parity_fuzz_seed440(gpu):
    """SURVEY §8(d) D2 parity fuzz: seed 440, message length 0..600, random
    sub-ranges crossing 10^k and ranges ending at 2^64-1."""
    rng = random.Random(440)
    for i in range(60):
        m = bytes(rng.randrange(0, 256) for _ in range(rng.randrange(0, 601)))
        if i % 4 == 3:
            hi = U64
            lo = hi - rng.randrange(0, 40_000)
        else:
            c = 10 ** rng.randrange(1, 20)
            lo = max(0, c - rng.randrange(0, 20_000))
            hi = min(U64, c + rng.randrange(0, 20_000))
        exp = oracle.search(m, lo, hi, threads=8)
        for e in both_paths():
            with e:
                assert gpu.search(m, lo, hi) == exp, (len(m), lo, hi, e.kv)


def test_plan_invariance_small(gpu):
    """The result must not depend on how the range is cut into launches."""
    for m, lo, hi in ((b"cmu440", 0, 2_000_000), (b"x" * 60, 10 ** 9 - 7, 10 ** 9 + 600_000),
                      (b"a" * 100, 123, 345_678), (b"y" * 52, 10 ** 12 - 50_000, 10 ** 12 + 50_000)):
        exp = oracle.search(m, lo, hi, threads=8)
        for Ld in (1, 2, 3, 4, 5):
            for gb in (0, 1 << 20):
                for st, ft in ((1, 0), (2, 0), (2, 20_000), (1, 99_999)):
                    for q in (0, 1):  # one workgroup per chunk / work queue
                        with env(MINEHIP_LOWER_DIGITS=Ld, MINEHIP_MIN_LANES=1, MINEHIP_LAUNCH_NONCES=100_000,
                                 MINEHIP_GENERIC_BELOW=gb, MINEHIP_STREAMS=st, MINEHIP_FINE_TAIL=ft,
                                 MINEHIP_QUEUE=q):
                            assert gpu.search(m, lo, hi) == exp, (m[:8], Ld, gb, st, ft, q)
        # the tail split on the low-priority stream with tiny grids (many launches, partial-buffer
        # flushes on both streams)
        for st, ft, mb, q in ((2, 200_000, 3, 1), (2, 200_000, 3, 0)):
            with env(MINEHIP_LOWER_DIGITS=3, MINEHIP_MIN_LANES=1, MINEHIP_STREAMS=st, MINEHIP_FINE_TAIL=ft,
                     MINEHIP_QUEUE=q, MINEHIP_MAX_BLOCKS=mb):
                assert gpu.search(m, lo, hi) == exp, (m[:8], st, ft, mb, q)
        # tiny grids: many launches per bucket and many partial-buffer flushes (on both streams);
        # with one block per launch a search outruns the 4,096 work-queue counters, and the
        # launches past them run one workgroup per chunk
        for mb in (1, 3, 1000):
            for st in (1, 2):
                for q in (0, 1):
                    with env(MINEHIP_MAX_BLOCKS=mb, MINEHIP_MIN_LANES=1, MINEHIP_STREAMS=st, MINEHIP_QUEUE=q):
                        assert gpu.search(m, lo, hi) == exp, (m[:8], mb, st, q)


@pytest.mark.parametrize("msg,bits", [(b"cmu440", 32), (b"a" * 100, 34), (b"x" * 60, 34)])
def test_full_size_properties(gpu, msg, bits):
    """BASELINE configs[1] (2^32 nonces, single block) and configs[2]
    (long messages over 2^34: host midstate / two tail blocks)."""
    hi = (1 << bits) - 1
    r = gpu.search(msg, 0, hi)
    assert oracle.hash_(msg, r[1]) == r[0] and 0 <= r[1] <= hi  # re-hashes to itself
    with env(MINEHIP_STREAMS=1, MINEHIP_FINE_TAIL=0):  # one stream, no tail split
        assert gpu.search(msg, 0, hi) == r
    rng = random.Random(bits)
    for _ in range(2):  # split-range associativity
        mid = rng.randrange(1, hi)
        assert lexmin(gpu.search(msg, 0, mid), gpu.search(msg, mid + 1, hi)) == r
    with env(MINEHIP_LOWER_DIGITS=4, MINEHIP_MIN_LANES=1, MINEHIP_GENERIC_BELOW=0):
        assert gpu.search(msg, 0, hi) == r
    with env(MINEHIP_LOWER_DIGITS=1, MINEHIP_LAUNCH_NONCES=1 << 28):
        assert gpu.search(msg, 0, hi) == r
    assert gpu.search_multi(msg, 0, hi, devs=[0, 0, 0], chunk=(1 << bits) // 7 + 3) == r
    # no sampled nonce beats it (oracle on 200k random nonces of the range)
    sample = np.random.default_rng(bits).integers(0, hi, size=200_000, dtype=np.uint64, endpoint=True)
    hs = oracle.hash_batch(msg, sample)
    assert int(hs.min()) >= r[0]


def test_miner_handle(gpu):
    req = gpu.marshal(gpu.NewRequest("cmu440", 0, 9999999))
    res = gpu.miner_handle(req)
    assert res == b'{"Type":2,"Data":"","Lower":0,"Upper":0,"Hash":1228377698034,"Nonce":1067492}'
    assert gpu.unmarshal(res) == gpu.NewResult(1228377698034, 1067492)


def test_search_multi_matches(gpu):
    for m, lo, hi in ((b"cmu440", 5, 3_000_000), (b"z" * 70, U64 - 2_000_000, U64)):
        exp = gpu.search(m, lo, hi)
        assert gpu.search_multi(m, lo, hi, devs=[0, 0], chunk=123_457) == exp
        assert gpu.search_multi(m, lo, hi, devs=[0]) == exp


def test_profile_counters(gpu):
    gpu.profile_enable(0, True)
    gpu.search("cmu440", 0, (1 << 30) - 1)
    p = gpu.profile_read(0)
    gpu.profile_enable(0, False)
    plan = gpu.plan("cmu440", 0, (1 << 30) - 1)
    fast = [q for q in plan if q["kind"] == 0]
    assert p["fast_launches"] == len(fast) and p["fast_ns"] > 0
    assert p["fast_nonces"] + p["generic_nonces"] == 1 << 30
    assert p["fast_ops"] == sum(q["count"] * q["nonce_ops"] for q in fast)
    assert p["fast_slots"] == sum(q["count"] * q["nonce_slots"] for q in fast)
    ks = gpu.profile_kernels(0)  # still readable after profile_enable(0, False)
    assert sum(k["launches"] for k in ks) == p["fast_launches"]
    assert sum(k["nonces"] for k in ks) == p["fast_nonces"]
    assert sum(k["ops"] for k in ks) == p["fast_ops"]
    assert abs(sum(k["ns"] for k in ks) - p["fast_ns"]) <= len(ks)
    assert {(k["word"], k["mode"]) for k in ks} == {(q["word"], q["mode"]) for q in fast}


def test_fast_kernels_run_from_the_embedded_module(gpu):
    """fast_search<J, MODE> runs from the code object embedded in libminehip.so (the issue-priority
    build).  In the dev build (the same sources plus hooks, run in a child process),
    pointing MINEHIP_DEV_CODE_OBJECT at a missing file makes a fast search fail loudly -- nothing
    falls back to another copy of the kernels -- and the embedded module serves the next search
    again.  The product library has no such hook (test_abi.py::test_product_library_has_no_dev_hooks)."""
    from conftest import run_dev
    lo = 10 ** 9
    r = run_dev(f"""
import os, minehip
assert minehip.LIB_PATH.endswith("build/dev/libminehip.so"), minehip.LIB_PATH
os.environ["MINEHIP_DEV_CODE_OBJECT"] = "/nonexistent/fast_search.hsaco"
try:
    minehip.search(b"cmu440", {lo}, {lo + (1 << 24) - 1})
    raise SystemExit("fast search ran without its code object")
except minehip.MinehipError as e:
    assert e.code == minehip.MH_EHIP, e
del os.environ["MINEHIP_DEV_CODE_OBJECT"]
print(*minehip.search(b"cmu440", {lo}, {lo + 199_999}))
""")
    assert r.returncode == 0, r.stderr[-2000:]
    got = tuple(int(x) for x in r.stdout.split()[-2:])
    assert got == oracle.search(b"cmu440", lo, lo + 199_999, threads=4)


@pytest.mark.gpu
def test_code_object_without_queue_marker_runs_static(gpu):
    """A code object loaded through the dev build's MINEHIP_DEV_CODE_OBJECT hook without the
    work-queue marker (as one built from pre-queue sources) runs one workgroup per chunk -- every
    chunk searched, whatever the launch's resident grid -- and gives the product's answer
    (build/fast_search_nomarker.hsaco: the same kernels, marker removed)."""
    from conftest import run_dev
    co = os.path.join(ROOT, "build", "fast_search_nomarker.hsaco")
    assert os.path.exists(co), "make all builds it"
    lo, hi = 10 ** 9, 10 ** 9 + (1 << 30) - 1  # ~1,000 chunks of fast_search<4, One> at L = 3
    exp = gpu.search(b"cmu440", lo, hi)
    r = run_dev(f"import minehip; print(*minehip.search(b'cmu440', {lo}, {hi}))",
                MINEHIP_DEV_CODE_OBJECT=co, MINEHIP_MIN_LANES=1)
    assert r.returncode == 0, r.stderr[-2000:]
    assert tuple(int(x) for x in r.stdout.split()[-2:]) == exp
