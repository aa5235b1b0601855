"""CPU tests of the C-ABI library: load, exports, argument/error behaviour,
the launch planner (host-only) and the bitcoin.Message codec.  No GPU compute
is called here."""
import ctypes
import os
import random
import re

import pytest

import minehip
from minehip import _lib
from conftest import ROOT

U64 = (1 << 64) - 1


def header_symbols():
    inc = os.path.join(ROOT, "include")
    src = "".join(open(os.path.join(inc, f)).read() for f in sorted(os.listdir(inc)) if f.endswith(".h"))
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mh_[a-z_0-9]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    syms = header_symbols()
    assert set(syms) == set(_lib.EXPORTS)
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for s in syms:
        assert hasattr(raw, s), s


def test_product_library_has_no_dev_hooks():
    """The experiment and test hooks (code-object override, LDS cap, injected worker failure)
    exist only in the dev build (`make dev`), never in the package's library."""
    hooks = (b"MINEHIP_DEV_CODE_OBJECT", b"MINEHIP_DEV_LDS", b"MINEHIP_TEST_FAIL_WORKER", b"MINEHIP_TEST_SPAWN_LIMIT")
    prod = open(_lib.PRODUCT_LIB_PATH, "rb").read()
    assert not [h for h in hooks if h in prod]
    from conftest import DEV_LIB
    if os.path.exists(DEV_LIB):
        dev = open(DEV_LIB, "rb").read()
        assert all(h in dev for h in hooks)
    # and the package loads the product library unless told otherwise
    if not os.environ.get("MINEHIP_LIB"):
        assert _lib.LIB_PATH == _lib.PRODUCT_LIB_PATH


def test_abi_version_and_devices():
    hdr = open(os.path.join(ROOT, "include", "minehip.h")).read()
    v = int(re.search(r"#define MH_ABI_VERSION (\d+)", hdr).group(1))
    assert minehip.lib.mh_abi_version() == v == _lib.MH_ABI_VERSION == 5
    assert minehip.device_count() >= 0


def test_binding_refuses_another_abi(tmp_path):
    """_lib refuses a library whose mh_abi_version differs from the binding's: its
    structs would be read at other strides."""
    src = tmp_path / "fake.c"
    src.write_text("int mh_abi_version(void) { return 3; }\n")
    so = tmp_path / "libfake.so"
    import subprocess
    import sys
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    r = subprocess.run([sys.executable, "-c", "import minehip"], capture_output=True, text=True,
                       env=dict(os.environ, MINEHIP_LIB=str(so),
                                PYTHONPATH=os.path.join(ROOT, "bitcoin-miner_amd")))
    assert r.returncode != 0 and "has ABI 3" in r.stderr, r.stderr[-500:]


def test_no_device_fails_loudly():
    if minehip.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(minehip.MinehipError) as e:
        minehip.search("cmu440", 0, 10)
    assert e.value.code == minehip.MH_ENODEV
    with pytest.raises(minehip.MinehipError):
        minehip.hash_batch("cmu440", [1, 2, 3])


def test_argument_errors():
    h = ctypes.c_uint64()
    n = ctypes.c_uint64()
    rc = minehip.lib.mh_search(0, b"x", 1, 5, 4, ctypes.byref(h), ctypes.byref(n))
    assert rc == minehip.MH_ERANGE
    rc = minehip.lib.mh_search(0, b"x", 1, 0, 4, None, ctypes.byref(n))
    assert rc == minehip.MH_EINVAL
    assert b"NULL" in minehip.lib.mh_last_error()
    rc = minehip.lib.mh_search(0, None, 3, 0, 4, ctypes.byref(h), ctypes.byref(n))
    assert rc == minehip.MH_EINVAL
    with pytest.raises(minehip.MinehipError) as e:
        minehip.plan("x", 9, 3)
    assert e.value.code == minehip.MH_ERANGE


# ---- planner ---------------------------------------------------------------

def digits(n):
    return len(str(n))


def check_plan(msg, lo, hi):
    pieces = minehip.plan(msg, lo, hi)
    assert pieces, "empty plan"
    cur = lo
    plen = len(msg) + 1
    for p in pieces:
        assert p["first"] == cur, (msg, lo, hi, p)
        assert p["count"] >= 1
        last = p["first"] + p["count"] - 1
        assert last <= hi
        d = p["digits"]
        t = plen % 64
        assert digits(p["first"]) == d, p
        if p["kind"] == 1:  # generic: may span buckets (coalesced); blocks of its longest nonce
            assert p["count"] <= (1 << 17) * 256  # PlanOpts.max_blocks workgroups of 256
            assert p["blocks"] == (1 if t + digits(last) + 9 <= 64 else 2)
        else:               # fast: one decimal bucket
            assert digits(last) == d, p
            assert p["blocks"] == (1 if t + d + 9 <= 64 else 2)
        if p["kind"] == 0:
            L = p["lo_digits"]
            R = 10 ** L
            assert 1 <= L <= min(5, d - 1)
            assert p["first"] % R == 0 and p["count"] % R == 0  # whole runs only
            pl = t + d - 1
            base = 64 if (p["blocks"] == 2 and pl >= 64) else 0
            mode = p["mode"] % 3
            if p["mode"] < 3:
                assert p["word"] == (pl - base) >> 2
                assert ((pl - base - L + 1) >> 2) >= p["word"] - 1
            else:  # Early: the innermost digit ends word J, the word before the last digit's
                assert p["word"] == ((pl - base) >> 2) - 1
                pos = pl - (base + 4 * p["word"] + 3)  # its decimal position; the group's: pos+1..
                assert 1 <= pos and pos + L <= d and pl - pos - (L - 1) >= max(t, base)
                block = 10 ** (pos + L)
                assert p["first"] % block == 0 and p["count"] % block == 0  # whole blocks of lanes
            if mode == 1:
                assert pl - L + 1 >= 64
            if mode == 2:
                assert pl < 64 and 13 <= p["word"] + (p["mode"] >= 3) <= 15
        cur = last + 1
    assert cur - 1 == hi
    return pieces


def test_plan_covers_exactly():
    rng = random.Random(440)
    msgs = [b"", b"cmu440", b"x" * 54, b"x" * 55, b"x" * 60, b"a" * 100, b"y" * 127, b"z" * 600]
    msgs += [bytes(rng.choice(b"abc ") for _ in range(L)) for L in range(0, 130, 3)]
    for m in msgs:
        check_plan(m, 0, 2 ** 32 - 1)
        check_plan(m, 0, 0)
        check_plan(m, U64 - 12345, U64)
        check_plan(m, U64, U64)
        for _ in range(4):
            k = rng.randrange(1, 20)
            lo = max(0, 10 ** k - rng.randrange(0, 10 ** min(k, 6)))
            hi = min(U64, lo + rng.randrange(0, 10 ** 7))
            check_plan(m, lo, hi)


def test_plan_fine_tail_covers_exactly(monkeypatch):
    """MINEHIP_FINE_TAIL: the last runs of each full-L bucket are re-planned at L - 1 (a piece of
    100-nonce lanes); the plan still tiles the range exactly, for every layout."""
    monkeypatch.setenv("MINEHIP_FINE_TAIL", str(1 << 28))
    for m in (b"cmu440", b"x" * 60, b"a" * 100, b"y" * 52, b"z" * 62):
        pieces = check_plan(m, 0, 2 ** 34 - 1)
        coarse = {p["digits"] for p in pieces if p["kind"] == 0 and p["lo_digits"] == 3}
        tails = [p for p in pieces if p["kind"] == 0 and p["lo_digits"] == 2 and p["digits"] in coarse]
        assert tails and all(p["count"] <= 1 << 28 for p in tails)
        check_plan(m, 549755813888, 549755813888 + 6871947673)
        check_plan(m, U64 - (1 << 33), U64)


def test_plan_early_layouts_tile_and_cost_less(monkeypatch):
    """MINEHIP_EARLY (default 1): where the last digit sits in word 1, 9 or 14, a bucket's fast
    pieces enumerate the digit ending the word before it innermost (fast_search<J, 3..5>); the
    lanes of one block then interleave (innermost digit at decimal position p >= L), pieces are
    whole blocks, and the plan still tiles the range exactly -- at a lower algorithmic cost than
    the last-digit plan of the same range."""
    cases = ((b"x" * 60, 0, 2 ** 34 - 1, {(0, 4)}),                       # configs[2], two tail blocks
             ((b"cmu440-" * 10)[:30], 0, 2 ** 32 - 1, {(8, 3)}),          # <9, One> -> <8, OneEarly>
             ((b"cmu440-" * 10)[:48], 0, 2 ** 32 - 1, {(13, 5)}),         # <14, Two> -> <13, TwoEarly>
             (b"", 10 ** 6, 10 ** 7 - 1, {(0, 3)}))                        # d = 7: last digit in word 1
    for m, lo, hi, early in cases:
        cost = {}
        for e in (1, 0):
            monkeypatch.setenv("MINEHIP_EARLY", str(e))
            pieces = check_plan(m, lo, hi)
            modes = {(p["word"], p["mode"]) for p in pieces if p["kind"] == 0}
            assert (modes >= early) if e else not any(md >= 3 for _, md in modes), (m[:8], e, modes)
            cost[e] = sum(p["count"] * p["nonce_ops"] for p in pieces if p["kind"] == 0)
            check_plan(m, U64 - (1 << 33), U64)
        assert cost[1] < cost[0] * 0.995, (m[:8], cost)


def test_plan_early_every_position_tiles():
    """The ranges test_gpu_parity.py::test_early_layout_every_position runs on the GPU (every
    Early kernel x innermost position p = 1..4 x L = 1..3, the u64 top included) are planned as
    exact tilings of whole blocks."""
    from test_gpu_parity import early_position_cases, env
    cases = early_position_cases()
    assert {(k[0], k[1], k[2]) for k in cases} >= {(j, m, p) for j, m in ((8, 3), (0, 4), (13, 5))
                                                     for p in (1, 2, 3, 4)}
    for (m, lo, hi, Ld) in cases.values():
        with env(MINEHIP_LOWER_DIGITS=Ld, MINEHIP_MIN_LANES=1, MINEHIP_GENERIC_BELOW=0):
            check_plan(m, lo, hi)


def test_plan_uses_fast_kernel_for_bulk():
    pieces = check_plan(b"cmu440", 0, 2 ** 32 - 1)
    fast = sum(p["count"] for p in pieces if p["kind"] == 0)
    assert fast / 2 ** 32 > 0.999  # [0, 10^6) is one generic launch
    # long message, digits in the second tail block: per-run prefix block
    pieces = check_plan(b"x" * 60, 0, 2 ** 34 - 1)
    assert {p["mode"] for p in pieces if p["kind"] == 0} >= {1}
    assert sum(p["count"] for p in pieces if p["kind"] == 0) / 2 ** 34 > 0.9999


def test_plan_coalesces_small_buckets():
    # [0, 10^7): buckets d = 1..6 (10^6 nonces) in one generic launch, d = 7 fast
    pieces = check_plan(b"cmu440", 0, 10 ** 7 - 1)
    assert [(p["kind"], p["first"], p["count"]) for p in pieces] == [(1, 0, 10 ** 6), (0, 10 ** 6, 9 * 10 ** 6)]
    # consecutive pieces never both generic (they would have been coalesced) unless one is full
    for m in (b"", b"x" * 60, b"a" * 100):
        ps = check_plan(m, 0, 2 ** 34 - 1)
        for a, b in zip(ps, ps[1:]):
            assert not (a["kind"] == 1 and b["kind"] == 1 and a["count"] < 65536 * 256)


def test_plan_launch_cap():
    """PlanOpts: at most 2^35 nonces and 131,072 workgroups of 256 lanes per fast launch, and
    configs[3]'s big buckets run 1,000-nonce lanes (L = 3) in launches near the cap, each
    bucket ending in one tail piece of <= 2^28 nonces at L = 2 (the default fine_tail)."""
    pieces = check_plan(b"cmu440", 0, 2 ** 40 - 1)
    fast = [p for p in pieces if p["kind"] == 0]
    assert max(p["count"] for p in pieces) <= 2 ** 35
    for p in fast:
        assert -(-(p["count"] // 10 ** p["lo_digits"]) // 256) <= 131072
    for d in (11, 12, 13):
        b = [p for p in fast if p["digits"] == d]
        assert [p["lo_digits"] for p in b] == [3] * (len(b) - 1) + [2]
        assert b[-1]["count"] <= 2 ** 28 and b[-1]["count"] > 2 ** 27
        assert max(p["count"] for p in b) > 2 ** 34


# ---- bitcoin.Message codec (Go encoding/json bytes) ------------------------

GO_JSON = [
    (minehip.NewJoin(), b'{"Type":0,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}'),
    (minehip.NewRequest("cmu440", 0, 9999999),
     b'{"Type":1,"Data":"cmu440","Lower":0,"Upper":9999999,"Hash":0,"Nonce":0}'),
    (minehip.NewResult(1228377698034, 1067492),
     b'{"Type":2,"Data":"","Lower":0,"Upper":0,"Hash":1228377698034,"Nonce":1067492}'),
    (minehip.NewRequest('a"b\\c\n\t\r<>&\x01', 0, U64),
     b'{"Type":1,"Data":"a\\"b\\\\c\\n\\t\\r\\u003c\\u003e\\u0026\\u0001","Lower":0,'
     b'"Upper":18446744073709551615,"Hash":0,"Nonce":0}'),
    (minehip.NewRequest("héllo ✓ 世 ", 1, 2),
     '{"Type":1,"Data":"héllo ✓ 世\\u2028","Lower":1,"Upper":2,"Hash":0,"Nonce":0}'.encode()),
]


def test_marshal_matches_go():
    for m, js in GO_JSON:
        assert minehip.marshal(m) == js


def test_marshal_invalid_utf8():
    m = minehip.Message(minehip.Request, b"\xff\xfeok", 0, 1)
    assert minehip.marshal(m) == b'{"Type":1,"Data":"\\ufffd\\ufffdok","Lower":0,"Upper":1,"Hash":0,"Nonce":0}'


def test_unmarshal_roundtrip_and_go_rules():
    for m, js in GO_JSON:
        assert minehip.unmarshal(js) == m
    # case-insensitive keys, unknown keys, whitespace, escapes, key order
    m = minehip.unmarshal(b' { "upper" : 7 , "extra": [1, {"a": null}], "TYPE":1, "data":"x\\u00e9\\ud83d\\ude00",'
                          b' "lower":3 } ')
    assert m == minehip.Message(1, "xé\U0001F600", 3, 7)
    with pytest.raises(minehip.MinehipError):
        minehip.unmarshal(b'{"Type":1,"Lower":-1}')
    with pytest.raises(minehip.MinehipError):
        minehip.unmarshal(b'{"Lower":18446744073709551616}')
    with pytest.raises(minehip.MinehipError):
        minehip.unmarshal(b'not json')


def test_message_string():
    assert minehip.NewRequest("cmu440", 0, 9).String() == "[Request cmu440 0 9]"
    assert minehip.NewResult(5, 6).String() == "[Result 5 6]"
    assert minehip.NewJoin().String() == "[Join]"


def test_miner_handle_rejects_non_requests():
    # MH_ENOTREQ / MH_ERANGE are the codes a miner skips; anything else comes from the search
    # itself and makes the miner exit (INTEGRATION.md miner loop, csrc/apps/miner_main.cpp)
    with pytest.raises(minehip.MinehipError) as e:
        minehip.miner_handle(minehip.marshal(minehip.NewJoin()))
    assert e.value.code == minehip.MH_ENOTREQ
    with pytest.raises(minehip.MinehipError) as e:
        minehip.miner_handle(b"not json")
    assert e.value.code == minehip.MH_ENOTREQ
    with pytest.raises(minehip.MinehipError) as e:
        minehip.miner_handle(minehip.marshal(minehip.NewRequest("x", 9, 1)))
    assert e.value.code == minehip.MH_ERANGE


# fast_search<J, MODE>: One J = 0..13, Pre J = 0..4, Two J = 13..15, and the Early modes (the digit
# ending word J innermost) OneEarly J = 0, 8, PreEarly J = 0, TwoEarly J = 13
KERNELS = ({(j, 0) for j in range(14)} | {(j, 1) for j in range(5)} | {(13, 2), (14, 2), (15, 2)} |
           {(0, 3), (8, 3), (0, 4), (13, 5)})


KERNEL_CASE_NONCES = 250_000


def kernel_cases():
    """One (msg, lo, hi, early) per instantiated fast kernel (word J, mode), planned with
    MINEHIP_GENERIC_BELOW=0 (small buckets on the fast kernels) and MINEHIP_EARLY=early: the
    default (1) reaches the Early kernels, 0 the last-digit kernels they replace."""
    seen = {}
    old = {k: os.environ.get(k) for k in ("MINEHIP_GENERIC_BELOW", "MINEHIP_EARLY")}
    os.environ["MINEHIP_GENERIC_BELOW"] = "0"
    try:
        for early in (1, 0):
            os.environ["MINEHIP_EARLY"] = str(early)
            _kernel_cases(seen, early)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return seen


def _kernel_cases(seen, early):
    for L in range(0, 128):
        m = b"q" * L
        for d in range(2, 21):
            lo = 10 ** (d - 1)
            hi = min(U64, lo + KERNEL_CASE_NONCES)  # two blocks of an Early layout's lanes (<= 10^5 each)
            for p in minehip.plan(m, lo, hi):
                if p["kind"] == 0:
                    seen.setdefault((p["word"], p["mode"]), (m, lo, hi, early))


def test_every_instantiated_kernel_is_reachable():
    assert set(kernel_cases()) == KERNELS


def test_one_kernel_list():
    """layout.hpp's MH_FAST_KERNELS is the one list of fast_search layouts: the kernels
    fast_search.hip instantiates and the planner and the launcher accept (both call
    fast_kernel_exists over it), and the per-nonce loops csrc/loop_mix.py expects.  It is the set
    this file expects, and the embedded code object holds exactly its kernels."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "bitcoin-miner_amd", "csrc"))
    import loop_mix
    assert loop_mix.fast_kernels() == KERNELS
    from minehip import codeobj
    names = {k[".name"] for k in codeobj.metadata(codeobj.fast_code_object())["amdhsa.kernels"]}
    got = {tuple(int(x) for x in re.match(r"_ZN2mh11fast_searchILi(\d+)ELi(\d+)EE", n).groups())
           for n in names if "fast_search" in n}
    assert got == KERNELS
    src = {f: open(os.path.join(ROOT, "bitcoin-miner_amd", "csrc", f)).read()
           for f in ("plan.cpp", "search_kernels.hip", "fast_search.hip")}
    assert "return fast_kernel_exists(J, mode);" in src["plan.cpp"]
    assert "return fast_kernel_exists(J, mode);" in src["search_kernels.hip"]
    assert "MH_FAST_KERNELS(MH_INST)" in src["fast_search.hip"]


def test_embedded_code_object_carries_queue_marker():
    """The work queue is used only with a code object that carries fast_search.hip's
    mh_fast_queue_args marker at sizeof(FastArgs): the embedded object does, at the
    size of the kernels' FastArgs argument; the test artefact built without it does not."""
    from minehip import codeobj
    co = codeobj.fast_code_object()
    assert b"mh_fast_queue_args" in co
    md = codeobj.metadata(co)
    fast = [k for k in md["amdhsa.kernels"] if "fast_search" in k[".name"]]
    assert len(fast) == len(KERNELS)
    assert {k[".args"][0][".size"] for k in fast} == {520}      # FastArgs, by value
    nomarker = os.path.join(ROOT, "build", "fast_search_nomarker.hsaco")
    if os.path.exists(nomarker):
        assert b"mh_fast_queue_args" not in open(nomarker, "rb").read()
