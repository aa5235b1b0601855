"""Generate the full-size scan fixtures tests/golden/fullsize_<cfg>.json.

TEST INFRASTRUCTURE.  BASELINE.json's configs scan 2^32..2^35 nonces, far more
than the per-nonce oracle restatement finishes in a test.  This script scans
them once, here, with OpenSSL's SHA-256 (tests/golden/fullsize_scan.c,
libcrypto 3, SHA-NI) and records the (hash, nonce) minimum of every 2^24-nonce
chunk and of the whole range.  The GPU tests (tests/test_gpu_fullsize.py) then
check the HIP path bit-exact at full size, chunk by chunk and whole, and
bench.py checks its own result against the same file.

Independence: OpenSSL is neither our kernel nor oracle/sha256_oracle.c.  As a
cross-check this script also rescans sample chunks with Python hashlib (the
generator of tests/golden/gen_golden.py) and with the C oracle, and fails if
any answer differs.

Configs (BASELINE.json configs):
  cfg2   "cmu440", [0, 2^35-1]: configs[1] at N = 1 is [0, 2^32-1]; bench.py's
         weak-scaling shards at N = 2/4/8 are [0, N*2^32-1], all covered.
  cfg3a  "a" * 100, [0, 2^34-1]: configs[2], host-midstate block.
  cfg3b  "x" * 60,  [0, 2^34-1]: configs[2], two tail blocks.
  two13, two14, two15, pre0, pre2
         (b"cmu440-" repeated)[:n] for n = 45, 48, 52, 55, 62, [0, 2^32-1]: the
         tail layouts BASELINE's messages do not reach at d = 10 -- the last digit
         in word 13 / 14 / 15 of a tail block that spills into a second block
         (fast_search<J, kModeTwo>), or in word 0 / 2 of the second tail block
         (kModePre; cfg3b covers word 1).  The lower buckets of each range go
         through other layouts (kModeOne, smaller J), all at full size.
  one1, one5, one7, one8, one10, one12
         (b"cmu440-" repeated)[:n] for n = 0, 13, 21, 25, 30, 41, [0, 2^32-1]: one tail
         block, the d = 7..10 buckets in fast_search<1|2|5|7|8|9|10|12, One>; with
         cfg2 (<3>, <4>), cfg3a (<11>), two13's lower buckets (<13>) and top (<6>)
         every layout the default plan sends to the fast kernels has a fixture
  pre3, pre4, top
         2^32 nonces from 10^13 / 10^17 for the 62-byte message (the 14- and
         18-digit buckets: fast_search<3, Pre>, <4, Pre>), and "cmu440" over
         [2^64-2^32, 2^64-1] (20 digits, fast_search<6, One>, up to the last u64).
  cfg4s  "cmu440", 2^24-nonce samples of configs[3]/[4] ([0, 2^40-1] and
         [0, 2^42-1], digit buckets d = 11..13, too large to scan whole on a
         CPU): 96 seeded random chunks, the chunks straddling 10^11 and
         10^12, and the last chunks of [0, 2^40) and [0, 2^42).

Run:  python tests/golden/gen_fullsize.py [cfg ...]   (~15 min on 8 cores)
"""
import hashlib
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CHUNK_BITS = 24

CONFIGS = {
    "cfg2": (b"cmu440", 0, (1 << 35) - 1),
    "cfg3a": (b"a" * 100, 0, (1 << 34) - 1),
    "cfg3b": (b"x" * 60, 0, (1 << 34) - 1),
}
LAYOUTS = {"two13": 45, "two14": 48, "two15": 52, "pre0": 55, "pre2": 62}
for _name, _n in LAYOUTS.items():
    CONFIGS[_name] = ((b"cmu440-" * 10)[:_n], 0, (1 << 32) - 1)
for _name, _n in {"one1": 0, "one5": 13, "one7": 21, "one8": 25, "one10": 30, "one12": 41}.items():
    CONFIGS[_name] = ((b"cmu440-" * 10)[:_n], 0, (1 << 32) - 1)
CONFIGS["pre3"] = ((b"cmu440-" * 10)[:62], 10 ** 13, 10 ** 13 + (1 << 32) - 1)
CONFIGS["pre4"] = ((b"cmu440-" * 10)[:62], 10 ** 17, 10 ** 17 + (1 << 32) - 1)
CONFIGS["top"] = (b"cmu440", (1 << 64) - (1 << 32), (1 << 64) - 1)


def build(out_dir="/tmp/minehip_fullsize"):
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "fullsize_scan")
    subprocess.run(["gcc", "-O2", "-Wall", "-Wno-deprecated-declarations", "-o", exe,
                    os.path.join(HERE, "fullsize_scan.c"), "-lcrypto", "-lpthread"], check=True)
    return exe


def hashlib_scan(msg, lo, hi):
    base = hashlib.sha256(msg + b" ")
    best = None
    for n in range(lo, hi + 1):
        h = base.copy()
        h.update(str(n).encode())
        v = int.from_bytes(h.digest()[:8], "big")
        if best is None or v < best[0]:
            best = (v, n)
    return best


def sample_ranges():
    import random
    rng = random.Random(440)
    size = 1 << CHUNK_BITS
    los = {10 ** 11 - size // 2, 10 ** 12 - size // 2, (1 << 40) - size, (1 << 42) - size}
    while len(los) < 100:
        los.add(rng.randrange(1 << 35, (1 << 42) - size))
    return [(lo, lo + size - 1) for lo in sorted(los)]


def gen_samples(exe, threads, oracle):
    msg = b"cmu440"
    out = []
    for lo, hi in sample_ranges():
        r = subprocess.run([exe, msg.hex(), str(lo), str(hi), str(CHUNK_BITS - 3), str(threads)],
                           check=True, capture_output=True, text=True)
        out.append([lo, hi] + json.loads(r.stdout)["result"])
    for lo, hi, h, n in (out[0], out[-1]):
        assert oracle.search(msg, lo, hi, threads=threads) == (h, n)
    path = os.path.join(HERE, "fullsize_cfg4s.json")
    with open(path, "w") as f:
        json.dump({"msg_hex": msg.hex(), "chunk_bits": CHUNK_BITS, "samples": out,
                   "generator": "tests/golden/fullsize_scan.c (OpenSSL SHA-256), gen_fullsize.py",
                   "cross_checked": "first and last sample vs oracle/sha256_oracle.c"}, f, separators=(",", ":"))
        f.write("\n")
    print(f"cfg4s: {len(out)} samples -> {path}", flush=True)


def main(names):
    exe = build()
    threads = os.cpu_count() or 1
    sys.path.insert(0, ROOT)
    from oracle import oracle
    for name in names:
        if name == "cfg4s":
            gen_samples(exe, threads, oracle)
            continue
        msg, lo, hi = CONFIGS[name]
        t = time.time()
        r = subprocess.run([exe, msg.hex(), str(lo), str(hi), str(CHUNK_BITS), str(threads)],
                           check=True, capture_output=True, text=True)
        d = json.loads(r.stdout)
        dt = time.time() - t
        chunks = [tuple(c) for c in d["chunks"]]
        assert tuple(d["result"]) == min(chunks)
        # cross-checks: the first and last chunk with the C oracle, a 2^20 head of a
        # middle chunk with hashlib (whose answer must match that sub-scan's minimum)
        size = 1 << CHUNK_BITS
        for i in (0, len(chunks) - 1):
            c_lo = lo + i * size
            got = oracle.search(msg, c_lo, min(hi, c_lo + size - 1), threads=threads)
            assert got == chunks[i], (name, i, got, chunks[i])
        mid = len(chunks) // 2
        m_lo = lo + mid * size
        sub = subprocess.run([exe, msg.hex(), str(m_lo), str(m_lo + (1 << 20) - 1), "20", "1"],
                             check=True, capture_output=True, text=True)
        assert tuple(json.loads(sub.stdout)["result"]) == hashlib_scan(msg, m_lo, m_lo + (1 << 20) - 1)
        out = {
            "msg_hex": msg.hex(), "lo": lo, "hi": hi, "chunk_bits": CHUNK_BITS,
            "result": list(d["result"]), "chunks": [list(c) for c in chunks],
            "generator": "tests/golden/fullsize_scan.c (OpenSSL SHA-256), gen_fullsize.py",
            "cross_checked": "chunks 0 and last vs oracle/sha256_oracle.c; a 2^20 sub-range vs hashlib",
        }
        path = os.path.join(HERE, f"fullsize_{name}.json")
        with open(path, "w") as f:
            json.dump(out, f, separators=(",", ":"))
            f.write("\n")
        print(f"{name}: {len(chunks)} chunks, result {tuple(d['result'])}, {dt:.0f} s "
              f"({(hi - lo + 1) / dt / 1e6:.0f} MH/s on {threads} threads) -> {path}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or list(CONFIGS) + ["cfg4s"])
