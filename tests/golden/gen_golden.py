"""Generate the golden fixtures in tests/golden/ with Python hashlib.

hashlib is an independent FIPS 180-4 SHA-256 implementation (OpenSSL); the
reference's arithmetic is Go's crypto/sha256, which implements the same
standard.  The Go reference cannot run in this container (no Go toolchain),
so these fixtures plus the FIPS 180-4 published known answers (hard-coded
below, not generated) are what pin the oracle.

Semantics restated (reference /root/reference):
  Hash(msg, nonce) = BigEndian.Uint64(sha256("%s %d" % (msg, nonce))[:8])
      bitcoin/hash.go:13-17
  scan(msg, lo, hi) = lexicographic min of (Hash(msg, n), n) over n in
      [lo, hi] inclusive -- the strict-< first-minimum loop of the miner spec
      (reference stub bitcoin/miner/miner.go:33).

Run:  python tests/golden/gen_golden.py   (takes ~1 min; writes JSON files)
"""
import hashlib
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))

# FIPS 180-4 / NIST CSRC example values (published constants, not computed).
FIPS_KAT = [
    ("", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    ("abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    ("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    ("abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu",
     "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"),
    ("a" * 1000000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
]

U64 = (1 << 64) - 1


def go_hash(msg: bytes, nonce: int) -> int:
    d = hashlib.sha256(msg + b" " + str(nonce).encode()).digest()
    return int.from_bytes(d[:8], "big")


def scan(msg: bytes, lo: int, hi: int):
    base = hashlib.sha256(msg + b" ")
    best = None
    for n in range(lo, hi + 1):
        h = base.copy()
        h.update(str(n).encode())
        v = int.from_bytes(h.digest()[:8], "big")
        if best is None or v < best[0]:
            best = (v, n)
    return best


def edge_nonces():
    s = {0, 1, 2, 9, 10, 11, 99, 100, 101, (1 << 32) - 1, 1 << 32, (1 << 32) + 1,
         (1 << 63) - 1, 1 << 63, U64 - 1, U64, 4294967295, 9999999, 1067492}
    for k in range(1, 20):
        s.update({10 ** k - 1, 10 ** k, 10 ** k + 1})
    return sorted(x for x in s if 0 <= x <= U64)


def messages():
    rng = random.Random(440)
    msgs = [b"", b"cmu440", b"a", b"x" * 55, b"x" * 60, b"a" * 100, b"hello world",
            "héllo ✓ 世界".encode(), bytes(range(1, 64)), b"\x00\xff\x80 \x00"]
    # every prefix length modulo 64 (tail offset) is a distinct kernel layout
    for L in list(range(0, 130)) + [191, 192, 193, 255, 256, 300, 447, 600, 601, 602, 603]:
        msgs.append(bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz0123456789 ") for _ in range(L)))
    seen, out = set(), []
    for m in msgs:
        if m not in seen:
            seen.add(m)
            out.append(m)
    return out


def main():
    for m, hx in FIPS_KAT:
        assert hashlib.sha256(m.encode()).hexdigest() == hx, m[:16]
    rng = random.Random(440)
    fips = [{"msg_hex": m.encode().hex(), "sha256": hx} for m, hx in FIPS_KAT if len(m) < 4096]
    fips_million_a = FIPS_KAT[-1][1]

    hv = []
    edges = edge_nonces()
    for m in messages():
        nonces = list(edges) + [rng.getrandbits(64) for _ in range(6)] + [rng.randrange(10 ** 6) for _ in range(4)]
        for n in nonces:
            hv.append([m.hex(), str(n), str(go_hash(m, n))])

    sv = []
    cases = [
        (b"cmu440", 0, 9999), (b"cmu440", 0, 999999), (b"cmu440", 0, 0), (b"cmu440", 5, 5),
        (b"cmu440", 9990, 10010), (b"cmu440", 99990, 100009), (b"cmu440", U64 - 5000, U64),
        (b"cmu440", (1 << 32) - 3000, (1 << 32) + 3000), (b"cmu440", 10 ** 19 - 2000, 10 ** 19 + 2000),
        (b"", 0, 20000), (b"x" * 60, 0, 99999), (b"a" * 100, 123456, 223456), (b"x" * 55, 0, 30000),
        (b"x" * 54, 0, 30000), (b"x" * 50, 999000, 1001000), (b"x" * 119, 0, 30000),
        ("héllo ✓ 世界".encode(), 7, 5007), (b"a" * 600, 0, 5000), (b"tie", 0, 3),
    ]
    for _ in range(12):  # seed-440 fuzz: random msg length, random ranges crossing 10^k
        L = rng.randrange(0, 601)
        m = bytes(rng.choice(b"abcdefghijklmnopqrstuvwxyz ") for _ in range(L))
        k = rng.randrange(1, 20)
        c = 10 ** k
        lo = max(0, c - rng.randrange(1, 3000))
        cases.append((m, lo, min(U64, lo + rng.randrange(0, 6000))))
    for m, lo, hi in cases:
        h, n = scan(m, lo, hi)
        sv.append({"msg_hex": m.hex(), "lower": str(lo), "upper": str(hi), "hash": str(h), "nonce": str(n)})

    # the config-1 answer (BASELINE.json configs[0]): 10^7 nonces, ~10 s
    h, n = scan(b"cmu440", 0, 9999999)
    big = [{"msg_hex": b"cmu440".hex(), "lower": "0", "upper": "9999999", "hash": str(h), "nonce": str(n)}]

    with open(os.path.join(HERE, "fips180_4.json"), "w") as f:
        json.dump({"vectors": fips, "million_a": fips_million_a}, f, indent=1)
    with open(os.path.join(HERE, "hash_vectors.json"), "w") as f:
        json.dump({"fields": ["msg_hex", "nonce", "hash"], "vectors": hv}, f, separators=(",", ":"))
    with open(os.path.join(HERE, "scan_vectors.json"), "w") as f:
        json.dump({"small": sv, "config1": big}, f, indent=1)
    print(len(fips), "fips,", len(hv), "hash vectors,", len(sv), "scan vectors, config1", big[0])


if __name__ == "__main__":
    main()
