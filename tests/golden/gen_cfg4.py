"""Generate tests/golden/fullsize_cfg4.json: BASELINE configs[3] whole.

TEST INFRASTRUCTURE.  configs[3] scans "cmu440" over [0, 2^40-1] (~1.1e12
nonces).  [0, 2^35-1] is already in fullsize_cfg2.json (OpenSSL scan, 2^24
chunks); this script adds [2^35, 2^40-1], scanned here on the CPU with
tests/golden/shani_scan.c (x86 SHA extensions, 2^28-nonce chunks, ~3 h on 8
cores, resumable), and writes the minimum of every 2^32-nonce chunk of
[0, 2^40-1] and of the whole range.

Before its answers are used, shani_scan is checked against OpenSSL:
  * every fullsize_cfg4s.json sample chunk inside [2^35, 2^40) (2^24 nonces
    each, d = 11..13, incl. the chunk straddling 10^11 and the last one below
    2^40), rescanned by shani_scan;
  * 64 of fullsize_cfg2.json's 2^24-chunk minima (OpenSSL), rescanned;
  * each 2^28 chunk line of the scan is checked to tile [2^35, 2^40) exactly.

Run:  python tests/golden/gen_cfg4.py [--scan-file F] [--threads T]
      (the scan appends to F and skips chunks already in it)
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
MSG = b"cmu440"
LO, HI = 1 << 35, (1 << 40) - 1
SCAN_BITS = 28
OUT_BITS = 32


def build(out_dir="/tmp/minehip_cfg4"):
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "shani_scan")
    subprocess.run(["gcc", "-O3", "-Wall", "-o", exe, os.path.join(HERE, "shani_scan.c"), "-lpthread"],
                   check=True)
    return exe


def shani(exe, lo, hi, bits, threads):
    out = subprocess.run([exe, MSG.hex(), str(lo), str(hi), str(bits), str(threads)], check=True,
                         capture_output=True, text=True).stdout
    return sorted(tuple(int(x) for x in ln.split()) for ln in out.splitlines())


def check_against_openssl(exe, threads):
    d4s = json.load(open(os.path.join(HERE, "fullsize_cfg4s.json")))
    n = 0
    for lo, hi, h, nn in d4s["samples"]:
        if lo >= LO and hi <= HI:
            got = shani(exe, lo, hi, 24, threads)
            assert len(got) == 1 and got[0][2:] == (h, nn), (lo, hi, got, h, nn)
            n += 1
    d2 = json.load(open(os.path.join(HERE, "fullsize_cfg2.json")))
    size = 1 << d2["chunk_bits"]
    picks = list(range(0, len(d2["chunks"]), len(d2["chunks"]) // 64))[:64]
    for i in picks:
        a = d2["lo"] + i * size
        got = shani(exe, a, a + size - 1, d2["chunk_bits"], threads)
        assert got[0][2:] == tuple(d2["chunks"][i]), (i, got, d2["chunks"][i])
    return n, len(picks)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scan-file", default="/tmp/minehip_cfg4/cfg4_done.txt")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    args = ap.parse_args()
    exe = build()
    ns, nc = check_against_openssl(exe, args.threads)
    print(f"shani_scan == OpenSSL on {ns} cfg4s samples and {nc} cfg2 chunks", file=sys.stderr)
    if not os.path.exists(args.scan_file):
        open(args.scan_file, "w").close()
    with open(args.scan_file, "a") as f:  # resumable: chunks already in the file are skipped
        subprocess.run([exe, MSG.hex(), str(LO), str(HI), str(SCAN_BITS), str(args.threads), args.scan_file],
                       check=True, stdout=f)
    rows = {}
    for ln in open(args.scan_file):
        lo, hi, h, n = (int(x) for x in ln.split())
        rows[lo] = (hi, h, n)
    los = sorted(rows)
    assert los[0] == LO and rows[los[-1]][0] == HI, "scan incomplete"
    assert all(rows[los[i]][0] + 1 == los[i + 1] for i in range(len(los) - 1)), "scan chunks do not tile"
    d2 = json.load(open(os.path.join(HERE, "fullsize_cfg2.json")))
    per = 1 << (OUT_BITS - d2["chunk_bits"])
    chunks = [min(tuple(c) for c in d2["chunks"][i:i + per]) for i in range(0, len(d2["chunks"]), per)]
    per = 1 << (OUT_BITS - SCAN_BITS)
    for i in range(0, len(los), per):
        chunks.append(min(rows[lo][1:] for lo in los[i:i + per]))
    assert len(chunks) == 1 << (40 - OUT_BITS)
    out = {
        "msg_hex": MSG.hex(), "lo": 0, "hi": HI, "chunk_bits": OUT_BITS,
        "result": list(min(chunks)),
        "source": "[0, 2^35): fullsize_cfg2.json (OpenSSL, 2^24 chunks); [2^35, 2^40): shani_scan.c "
                  "(x86 SHA extensions, 2^28 chunks), checked against OpenSSL by gen_cfg4.py",
        "chunks": [list(c) for c in chunks],
    }
    with open(os.path.join(HERE, "fullsize_cfg4.json"), "w") as f:
        json.dump(out, f)
    print(json.dumps(out["result"]))


if __name__ == "__main__":
    main()
