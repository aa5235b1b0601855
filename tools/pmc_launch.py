"""pmc_launch.py -- the process `bench.py` runs under `rocprofv3 --pmc` to
measure the HBM traffic of its dominant kernel (roofline.traffic).

One search of exactly the nonces the dominant fast_search launch covers in
the bench's own plan, so the counters of that dispatch are per launch:

  python tools/pmc_launch.py <msg> <lower> <upper> [dev]

No torch: only libminehip (ctypes), so the profiled process starts in ~1 s.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]


def main():
    import minehip
    msg = sys.argv[1].encode()
    lo, hi = int(sys.argv[2]), int(sys.argv[3])
    dev = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    print(minehip.search(msg, lo, hi, dev), flush=True)


if __name__ == "__main__":
    main()
