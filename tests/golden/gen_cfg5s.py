"""Generate tests/golden/fullsize_cfg5s.json: 64 sampled 2^28-nonce chunks of [2^40, 2^42-1], the
part of BASELINE configs[4] ("cmu440", [0, 2^42-1]) that fullsize_cfg4.json (the whole of
[0, 2^40)) does not cover.

TEST INFRASTRUCTURE.  A CPU scan of all 3 * 2^40 nonces would take ~9 h here; these 64 chunks
(2^34 nonces, ~4 min on 8 cores) sample it evenly: chunk i starts at 2^40 + i * 3 * 2^34 plus a
seeded jitter of whole 2^28 steps inside its 3 * 2^34 stride, so the samples spread over the
range without a pattern the kernel's launch layout could share, and the first and the last
2^28 chunk of the range are always in.  Every chunk is scanned with tests/golden/shani_scan.c
(x86 SHA extensions).  Before its answers are used, shani_scan is checked against OpenSSL
(tests/golden/fullsize_scan.c) on one of these very chunks, and through gen_cfg4's check
(fullsize_cfg4s.json samples and fullsize_cfg2.json chunks).

The GPU test (tests/test_gpu_fullsize.py::test_config5_sampled_chunks) searches every chunk and
checks that the answer chunk's minimum (fullsize_cfg5c.json, configs[4]'s result) beats every
sampled chunk's: the [2^40, 2^42) part of configs[4] pinned on the CPU by samples.

Run:  python tests/golden/gen_cfg5s.py [--threads T]
"""
import argparse
import json
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_cfg4  # noqa: E402  (build, shani, check_against_openssl)
import gen_fullsize  # noqa: E402  (build: the OpenSSL scanner)

MSG = b"cmu440"
LO, HI = 1 << 40, (1 << 42) - 1
BITS = 28
N = 64
OPENSSL_CHECK = 17  # the sample rescanned with OpenSSL


def sample_los(seed=5440):
    rng = random.Random(seed)
    size = 1 << BITS
    stride = (HI + 1 - LO) // N             # 3 * 2^34: a whole number of chunks
    los = [LO + i * stride + rng.randrange(stride // size) * size for i in range(N)]
    los[0], los[-1] = LO, HI + 1 - size      # the range's first and last chunk
    assert len(set(los)) == N and all(LO <= x and x + size - 1 <= HI and x % size == 0 for x in los)
    return los


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    exe = gen_cfg4.build()
    ns, nc = gen_cfg4.check_against_openssl(exe, a.threads)
    size = 1 << BITS
    samples = []
    for lo in sample_los():
        # 16 sub-chunks of 2^24 so that every thread works on a chunk; they must tile it
        got = gen_cfg4.shani(exe, lo, lo + size - 1, BITS - 4, a.threads)
        assert [r[:2] for r in got] == [(lo + (i << (BITS - 4)), lo + ((i + 1) << (BITS - 4)) - 1)
                                        for i in range(16)], got
        h, n = min(r[2:] for r in got)
        samples.append([lo, lo + size - 1, h, n])
    # the same chunk through OpenSSL's SHA-256 (an independent implementation)
    lo, hi, h, n = samples[OPENSSL_CHECK]
    ossl = gen_fullsize.build()
    r = subprocess.run([ossl, MSG.hex(), str(lo), str(hi), str(BITS - 4), str(a.threads)], check=True,
                       capture_output=True, text=True)
    assert tuple(json.loads(r.stdout)["result"]) == (h, n), (r.stdout[:200], h, n)
    print(f"shani_scan == OpenSSL on {ns} cfg4s samples, {nc} cfg2 chunks and sample {OPENSSL_CHECK}",
          file=sys.stderr)
    out = {
        "msg_hex": MSG.hex(), "lo": LO, "hi": HI, "chunk_bits": BITS,
        "source": f"shani_scan.c (x86 SHA extensions), {N} sampled 2^{BITS} chunks of [2^40, 2^42); "
                  f"sample {OPENSSL_CHECK} rescanned with OpenSSL (fullsize_scan.c) by gen_cfg5s.py",
        "samples": samples,
    }
    with open(os.path.join(HERE, "fullsize_cfg5s.json"), "w") as f:
        json.dump(out, f)
    print(json.dumps(min(s[2:] for s in samples)))


if __name__ == "__main__":
    main()
