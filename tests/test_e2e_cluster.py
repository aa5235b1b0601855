"""End-to-end rehearsal of BASELINE configs[4] with tools/cluster.py: a server,
miner processes and a client, with dropped-miner recovery.

The pieces are separate OS processes exchanging Go-JSON bitcoin.Messages over a
length-prefixed TCP framing on 127.0.0.1.  That framing stands in for the LSP
transport, which is Go, unchanged, and not in this image.  The server is the
library's mh_server loop.  One miner vanishes on receiving its first chunk;
the client's printed Result must still equal a direct scan of the whole range.

CPU: miners are tests/e2e_oracle_miner.py (the oracle, test infrastructure).
GPU: miners are `tools/cluster.py miner` (mh_miner_handle on cuda:0)."""
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT
from oracle import oracle

PY = sys.executable
CLUSTER = os.path.join(ROOT, "tools", "cluster.py")
ORACLE_MINER = os.path.join(ROOT, "tests", "e2e_oracle_miner.py")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_cluster(miners, msg, max_nonce, chunk, timeout):
    """miners: list of (argv builder(hostport) -> argv).  Returns the client's
    stdout and stderr; every process started here is killed afterwards."""
    port = free_port()
    hp = f"127.0.0.1:{port}"
    procs = []
    try:
        srv = [PY, CLUSTER, "server", str(port)] + (["--chunk", str(chunk)] if chunk else [])
        procs.append(subprocess.Popen(srv, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        for build in miners:
            procs.append(subprocess.Popen(build(hp), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        cl = subprocess.run([PY, CLUSTER, "client", hp, msg, str(max_nonce)], capture_output=True, text=True,
                            timeout=timeout)
        return cl.stdout.strip(), cl.stderr
    finally:
        for p in procs:  # exactly the processes started here, by PID
            p.kill()
            p.wait()


def oracle_miner(drop_after=0):
    return lambda hp: [PY, ORACLE_MINER, hp] + ([str(drop_after)] if drop_after else [])


def gpu_miner(drop_after=0):
    return lambda hp: [PY, CLUSTER, "miner", hp] + (["--drop-after", str(drop_after)] if drop_after else [])


def test_cluster_cpu_with_dropped_miner():
    out, err = run_cluster([oracle_miner(), oracle_miner(), oracle_miner(drop_after=1)],
                           "cmu440", 1_999_999, chunk=100_000, timeout=240)
    h, n = oracle.search("cmu440", 0, 1_999_999, threads=8)
    assert out == f"Result {h} {n}", err[-2000:]


@pytest.mark.gpu
def test_cluster_gpu_with_dropped_miner(gpu):
    max_nonce = (1 << 34) - 1
    out, err = run_cluster([gpu_miner(), gpu_miner(), gpu_miner(drop_after=1)],
                           "cmu440", max_nonce, chunk=1 << 30, timeout=600)
    h, n = gpu.search("cmu440", 0, max_nonce)
    assert out == f"Result {h} {n}", err[-2000:]
