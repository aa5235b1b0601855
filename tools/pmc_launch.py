"""pmc_launch.py -- the process `bench.py` runs under `rocprofv3 --pmc` to
measure the counters of its largest kernels (roofline.traffic, roofline.pmc).

One search per given range, each exactly the nonces one fast_search launch
covers in the bench's own plan, planned as that one launch (its lane length L,
one stream, no tail split), so the counters of those dispatches are per launch:

  python tools/pmc_launch.py <msg> <dev> <lower>:<upper>:<L> [<lower>:<upper>:<L> ...]

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
    os.environ.update(MINEHIP_STREAMS="1", MINEHIP_FINE_TAIL="0", MINEHIP_MIN_LANES="1")
    for r in sys.argv[3:]:
        lo, hi, L = (int(x) for x in r.split(":"))
        os.environ["MINEHIP_LOWER_DIGITS"] = str(L)
        fast = [p for p in minehip.plan(msg, lo, hi) if p["kind"] == 0]
        if len(fast) != 1 or (fast[0]["first"], fast[0]["count"], fast[0]["lo_digits"]) != (lo, hi - lo + 1, L):
            sys.exit(f"pmc_launch: [{lo}, {hi}] at L = {L} does not plan as one launch: {fast}")
        print(minehip.search(msg, lo, hi, dev), flush=True)


if __name__ == "__main__":
    main()
