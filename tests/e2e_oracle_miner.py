"""CPU miner for tests/test_e2e_cluster.py: the miner process of
bitcoin/miner/miner.go (join over LSP, Request -> scan -> Result) with the
test oracle in place of the GPU (test infrastructure only; the product miner
is bin/minehip-miner).  With DROP_AFTER = k it vanishes without a word on
receiving its k-th Request, like a crashed miner.

    python tests/e2e_oracle_miner.py HOST:PORT [DROP_AFTER]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]

import minehip  # noqa: E402
from minehip import lsp  # noqa: E402
from oracle import oracle  # noqa: E402


def params():
    p = lsp.NewParams()
    for env, f in (("LSP_EPOCH_LIMIT", "epoch_limit"), ("LSP_EPOCH_MILLIS", "epoch_millis"),
                   ("LSP_WINDOW_SIZE", "window_size")):
        if os.environ.get(env):
            setattr(p, f, int(os.environ[env]))
    return p


def main():
    drop_after = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    cl, err = lsp.NewClient(sys.argv[1], params())
    if err is not None:
        print("Failed to join with server:", err)
        return 1
    cl.Write(minehip.marshal(minehip.NewJoin()))
    seen = 0
    while True:
        payload, err = cl.Read()
        if err is not None:
            break
        m = minehip.unmarshal(payload)
        if m is None or m.Type != minehip.Request:
            continue
        seen += 1
        if seen == drop_after:
            os._exit(0)  # vanish: no Result, no Close
        cl.Write(minehip.marshal(minehip.NewResult(*oracle.search(m.Data, m.Lower, m.Upper, threads=2))))
    cl.Close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
