"""CPU miner for tests/test_e2e_cluster.py: tools/cluster.py's miner loop with
the test oracle in place of the GPU (test infrastructure only)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "tools"), os.path.join(ROOT, "bitcoin-miner_amd")]

import minehip  # noqa: E402
import cluster  # noqa: E402
from oracle import oracle  # noqa: E402


def handle(payload):
    m = minehip.unmarshal(payload)
    return minehip.marshal(minehip.NewResult(*oracle.search(m.Data, m.Lower, m.Upper, threads=2)))


if __name__ == "__main__":  # e2e_oracle_miner.py HOST:PORT [DROP_AFTER]
    cluster.miner(sys.argv[1], 0, handle, drop_after=int(sys.argv[2]) if len(sys.argv) > 2 else 0)
