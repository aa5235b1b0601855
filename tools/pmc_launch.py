"""pmc_launch.py -- the process `bench.py` runs under `rocprofv3 --pmc` to
measure the counters of its largest kernels (roofline.traffic, roofline.pmc).

One search per given range, each exactly the nonces one fast_search launch
covers in the bench's own plan, so the counters of those dispatches are per
launch:

  python tools/pmc_launch.py <msg> <dev> <lower>:<upper> [<lower>:<upper> ...]

No torch: only libminehip (ctypes), so the profiled process starts in ~1 s.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]


def main():
    import minehip
    msg = sys.argv[1].encode()
    dev = int(sys.argv[2])
    for r in sys.argv[3:]:
        lo, hi = (int(x) for x in r.split(":"))
        print(minehip.search(msg, lo, hi, dev), flush=True)


if __name__ == "__main__":
    main()
