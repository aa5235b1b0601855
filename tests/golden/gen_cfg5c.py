"""Generate tests/golden/fullsize_cfg5c.json: the 2^32-nonce chunk of BASELINE
configs[4] ("cmu440", [0, 2^42-1]) that holds its answer.

TEST INFRASTRUCTURE.  The GPU's configs[4] answer is (5743413, 4370581897648)
(profiles/r02ad_lsp_cfg4_8miners.json: 8 miner processes over LSP, equal to a
direct mh_search).  A CPU scan of all 2^42 nonces would take ~12 h here, so
this pins the answer's own chunk instead: [1017 * 2^32, 1018 * 2^32 - 1]
(d = 13), scanned with tests/golden/shani_scan.c (x86 SHA extensions; ~1 min on
8 cores) in 2^28-nonce chunks.  Before its answer is used, shani_scan is checked
against OpenSSL (gen_cfg4.check_against_openssl: every fullsize_cfg4s.json
sample chunk in [2^35, 2^40) and 64 fullsize_cfg2.json chunks) and on the
fullsize_cfg4s.json samples inside [2^40, 2^42).  The nonce 4370581897648 is
not an input here: the scan finds the chunk's minimum on its own.

Run:  python tests/golden/gen_cfg5c.py [--threads T]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_cfg4  # noqa: E402  (build, shani, check_against_openssl)

MSG = b"cmu440"
CHUNK = 1017
BITS = 28


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    exe = gen_cfg4.build()
    ns, nc = gen_cfg4.check_against_openssl(exe, a.threads)
    d4s = json.load(open(os.path.join(HERE, "fullsize_cfg4s.json")))
    nhi = 0
    for lo, hi, h, n in d4s["samples"]:
        if lo >= 1 << 40:
            got = gen_cfg4.shani(exe, lo, hi, 24, a.threads)
            assert len(got) == 1 and got[0][2:] == (h, n), (lo, hi, got, h, n)
            nhi += 1
    print(f"shani_scan == OpenSSL on {ns} + {nhi} cfg4s samples and {nc} cfg2 chunks", file=sys.stderr)
    lo, hi = CHUNK << 32, ((CHUNK + 1) << 32) - 1
    rows = gen_cfg4.shani(exe, lo, hi, BITS, a.threads)
    assert [r[0] for r in rows] == [lo + (i << BITS) for i in range(1 << (32 - BITS))], "chunks do not tile"
    assert all(r[1] == r[0] + (1 << BITS) - 1 for r in rows)
    chunks = [list(r[2:]) for r in rows]
    out = {
        "msg_hex": MSG.hex(), "lo": lo, "hi": hi, "chunk_bits": BITS,
        "result": list(min(tuple(c) for c in chunks)),
        "source": f"shani_scan.c (x86 SHA extensions, 2^{BITS} chunks), checked against OpenSSL by "
                  "gen_cfg5c.py; BASELINE configs[4]'s answer chunk",
        "chunks": chunks,
    }
    with open(os.path.join(HERE, "fullsize_cfg5c.json"), "w") as f:
        json.dump(out, f)
    print(json.dumps(out["result"]))


if __name__ == "__main__":
    main()
