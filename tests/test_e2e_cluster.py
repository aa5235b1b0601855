"""End-to-end BASELINE configs[4] layout over real LSP/UDP: the server, miner
and client processes of the reference (bitcoin/server, bitcoin/miner,
bitcoin/client), as separate OS processes
on 127.0.0.1, with dropped-miner recovery.

  server   bin/minehip-server <port>        libminehip's server loop over liblsp440
  miners   bin/minehip-miner <hostport>     GPU (mh_miner_handle), or on CPU
           tests/e2e_oracle_miner.py        the oracle over the same LSP
  client   bin/minehip-client <hostport> <msg> <maxNonce>

One miner disappears mid-job (it exits on its first Request, or is killed);
the server learns of it through LSP's epoch timeout (Read -> (connID, err),
the N3 fix) and hands its chunk to the others.  The client's printed Result
must equal a direct scan of [0, maxNonce].  LSP_EPOCH_MILLIS shortens epochs
so that loss is detected in ~0.5 s instead of EpochLimit x 2 s."""
import os
import socket
import subprocess
import sys
import time

import pytest

from conftest import PKG, ROOT
from oracle import oracle

PY = sys.executable
BIN = os.path.join(PKG, "bin")
ORACLE_MINER = os.path.join(ROOT, "tests", "e2e_oracle_miner.py")
ENV = dict(os.environ, LSP_EPOCH_MILLIS="100", LSP_EPOCH_LIMIT="5")


def free_udp_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_cluster(miners, msg, max_nonce, chunk, timeout, kill_after=None, tmp=None):
    """miners: argv builders (hostport -> argv).  kill_after = (index, seconds):
    SIGKILL that miner that long after the client starts.  Returns the client's
    stdout and the server's stderr.  Every process started here is killed by
    PID afterwards."""
    port = free_udp_port()
    hp = f"127.0.0.1:{port}"
    env = dict(ENV, MINEHIP_CHUNK=str(chunk)) if chunk else ENV
    err_path = os.path.join(tmp, "server.err")
    procs = []
    try:
        with open(err_path, "w") as serr:
            srv = subprocess.Popen([os.path.join(BIN, "minehip-server"), str(port)], stdout=subprocess.PIPE,
                                   stderr=serr, env=env, text=True)
            procs.append(srv)
            assert srv.stdout.readline().strip() == f"Server listening on port {port}"
            miner_procs = []
            for build in miners:
                p = subprocess.Popen(build(hp), stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env)
                procs.append(p)
                miner_procs.append(p)
            time.sleep(0.5)  # let the miners join before the Request
            cl = subprocess.Popen([os.path.join(BIN, "minehip-client"), hp, msg, str(max_nonce)],
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, text=True)
            procs.append(cl)
            if kill_after is not None:
                time.sleep(kill_after[1])
                miner_procs[kill_after[0]].kill()
            out, _ = cl.communicate(timeout=timeout)
        return out.strip(), open(err_path).read()
    finally:
        for p in procs:  # exactly the processes started here, by PID
            if p.poll() is None:
                p.kill()
            p.wait()


def oracle_miner(drop_after=0):
    return lambda hp: [PY, ORACLE_MINER, hp] + ([str(drop_after)] if drop_after else [])


def gpu_miner():
    return lambda hp: [os.path.join(BIN, "minehip-miner"), hp]


def test_usage_lines():
    r = subprocess.run([os.path.join(BIN, "minehip-client"), "x"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2 and r.stdout.startswith("Usage: ")
    r = subprocess.run([os.path.join(BIN, "minehip-client"), "127.0.0.1:1", "m", "-3"], capture_output=True,
                       text=True, timeout=30)
    assert r.stdout == "-3 is not a number.\n"
    r = subprocess.run([os.path.join(BIN, "minehip-server")], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2 and r.stdout.startswith("Usage: ")


def test_client_without_server_fails_to_connect():
    env = dict(ENV, LSP_EPOCH_MILLIS="50", LSP_EPOCH_LIMIT="2")
    r = subprocess.run([os.path.join(BIN, "minehip-client"), f"127.0.0.1:{free_udp_port()}", "cmu440", "9"],
                       capture_output=True, text=True, timeout=30, env=env)
    assert r.stdout == "Failed to connect to server: can not establish connection\n"


def test_client_sees_disconnected_when_server_dies(tmp_path):
    port = free_udp_port()
    srv = subprocess.Popen([os.path.join(BIN, "minehip-server"), str(port)], stdout=subprocess.PIPE,
                           stderr=subprocess.DEVNULL, env=ENV, text=True)
    try:
        srv.stdout.readline()
        cl = subprocess.Popen([os.path.join(BIN, "minehip-client"), f"127.0.0.1:{port}", "cmu440", "99"],
                              stdout=subprocess.PIPE, text=True, env=ENV)
        time.sleep(0.3)  # connected, Request sent; no miner, so no Result
        srv.kill()
        out, _ = cl.communicate(timeout=30)
        assert out == "Disconnected\n"
    finally:
        if srv.poll() is None:
            srv.kill()
        srv.wait()


def test_cluster_cpu_with_dropped_miner(tmp_path):
    out, err = run_cluster([oracle_miner(), oracle_miner(), oracle_miner(drop_after=1)],
                           "cmu440", 1_999_999, chunk=100_000, timeout=240, tmp=str(tmp_path))
    h, n = oracle.search("cmu440", 0, 1_999_999, threads=8)
    assert out == f"Result {h} {n}", err[-2000:]
    assert "lost" in err  # the server saw the dropped miner through LSP


def test_config0_full_range_over_lsp(tmp_path):
    """BASELINE configs[0]: the CPU miner over LSP on localhost, msg "cmu440", nonces
    0..9,999,999 in full -- the client prints the answer pinned in SURVEY §8(c) C4 and
    tests/golden/scan_vectors.json (hashlib), with one of three miners dropping mid-job."""
    out, err = run_cluster([oracle_miner(), oracle_miner(), oracle_miner(drop_after=1)],
                           "cmu440", 9_999_999, chunk=500_000, timeout=600, tmp=str(tmp_path))
    assert out == "Result 1228377698034 1067492", err[-2000:]
    assert "lost" in err


@pytest.mark.gpu
def test_cluster_gpu_with_killed_miner(gpu, tmp_path):
    # 3 GPU miner processes on the box's one GPU; one is SIGKILLed mid-job.
    max_nonce = (1 << 36) - 1
    out, err = run_cluster([gpu_miner(), gpu_miner(), gpu_miner()], "cmu440", max_nonce, chunk=1 << 31,
                           timeout=600, kill_after=(2, 1.0), tmp=str(tmp_path))
    h, n = gpu.search("cmu440", 0, max_nonce)
    assert out == f"Result {h} {n}", err[-2000:]
    assert "lost" in err and "requeued so far 0" not in err, err[-2000:]


def _server(tmp, env=ENV):
    port = free_udp_port()
    serr = open(os.path.join(tmp, "server.err"), "w")
    srv = subprocess.Popen([os.path.join(BIN, "minehip-server"), str(port)], stdout=subprocess.PIPE,
                           stderr=serr, env=env, text=True)
    assert srv.stdout.readline().strip() == f"Server listening on port {port}"
    return srv, port


def test_request_too_large_for_a_miner_frame_is_refused(tmp_path):
    """a client Request that fits one LSP datagram can grow past one when the server
    re-encodes it per miner chunk (Go's JSON escapes '<' as \\u003c: 6x).  The server refuses it up
    front and closes the client, which then sees its connection end (the minehip-client prints
    Disconnected), instead of the chunk write failing with LSP_ETOOBIG and the client waiting
    forever.  A Request just under the limit is still served."""
    from minehip import lsp
    import minehip
    srv, port = _server(str(tmp_path))
    try:
        miner, err = lsp.NewClient(f"127.0.0.1:{port}", lsp.NewParams(epoch_limit=5, epoch_millis=100))
        assert err is None
        assert miner.Write(minehip.marshal(minehip.NewJoin())) is None
        time.sleep(0.3)
        p = lsp.NewParams(epoch_limit=5, epoch_millis=100)
        # a non-Go client writes '<' raw: 14,000 bytes of Data, ~19 KB as one datagram
        big = b'{"Type":1,"Data":"' + b"<" * 14_000 + b'","Lower":0,"Upper":9}'
        cl, err = lsp.NewClient(f"127.0.0.1:{port}", p)
        assert err is None
        assert cl.Write(big) is None
        payload, err = cl.Read(timeout_ms=20_000)
        assert payload is None and err is not None        # closed by the server, no Result
        assert err.code in (lsp.LSP_ELOST, lsp.LSP_ECLOSED), err   # not a read timeout
        assert "too large" in open(os.path.join(str(tmp_path), "server.err")).read()
        cl.Close()
        # 7,000 '<' re-encode to 42 KB + bounds: one datagram (base64 ~ 56 KB < 65,507 B): served
        ok = b'{"Type":1,"Data":"' + b"<" * 7_000 + b'","Lower":0,"Upper":9}'
        cl, err = lsp.NewClient(f"127.0.0.1:{port}", p)
        assert cl.Write(ok) is None
        req, err = miner.Read(timeout_ms=20_000)
        assert err is None
        m = minehip.unmarshal(req)
        assert m.Type == minehip.Request and m.Data == b"<" * 7_000 and (m.Lower, m.Upper) == (0, 9)
        h, n = oracle.search(m.Data, 0, 9, threads=1)
        assert miner.Write(minehip.marshal(minehip.NewResult(h, n))) is None
        res, err = cl.Read(timeout_ms=20_000)
        assert err is None and minehip.unmarshal(res) == minehip.NewResult(h, n)
        cl.Close()
        miner.Close()
    finally:
        srv.kill()
        srv.wait()


# ---- BASELINE configs[4] at its stated size -----------------------------
CFG5_HI = (1 << 42) - 1
_cfg5 = {}


def _cfg5_direct(gpu):
    """One direct mh_search of configs[4]'s range (~90 s), shared by the tests below."""
    if "direct" not in _cfg5:
        _cfg5["direct"] = gpu.search(b"cmu440", 0, CFG5_HI)
    return _cfg5["direct"]


def _cfg5_checks(gpu, got):
    """configs[4]'s answer against everything that pins it without a CPU scan of 2^42 nonces."""
    from conftest import load_golden
    msg = b"cmu440"
    assert gpu.Hash(msg, got[1]) == got[0]                        # re-hashed by the generic kernel
    cfg4 = load_golden("fullsize_cfg4.json")                      # [0, 2^40-1] is a prefix of the range
    assert got <= tuple(cfg4["result"])
    s = load_golden("fullsize_cfg4s.json")                        # 100 OpenSSL-scanned 2^24 chunks
    assert all(got <= (h, n) for lo, hi, h, n in s["samples"] if hi <= CFG5_HI)
    c = load_golden("fullsize_cfg5c.json")                        # the answer's 2^32 chunk, SHA-NI scan
    assert c["lo"] <= got[1] <= c["hi"]
    assert got == tuple(c["result"])                              # the CPU-verified minimum of its chunk


@pytest.mark.gpu
def test_config5_direct_search(gpu):
    """BASELINE configs[4]'s range, "cmu440" over [0, 2^42-1], searched directly on one GPU."""
    _cfg5_checks(gpu, _cfg5_direct(gpu))


@pytest.mark.gpu
def test_config5_over_lsp_eight_gpu_miners_one_killed(gpu, tmp_path):
    """BASELINE configs[4] at its stated size: server + 8 GPU miner processes (configs[4]'s
    one-per-GPU layout; all on this box's GPU) + client over LSP/UDP, "cmu440" over
    [0, 2^42-1], one miner SIGKILLed 5 s in.  The client's Result equals the direct search,
    re-hashes, and is pinned by the fixtures (_cfg5_checks)."""
    out, err = run_cluster([gpu_miner()] * 8, "cmu440", CFG5_HI, chunk=None, timeout=480,
                           kill_after=(7, 5.0), tmp=str(tmp_path))
    assert out.startswith("Result "), err[-2000:]
    got = tuple(int(x) for x in out.split()[1:3])
    _cfg5_checks(gpu, got)
    assert got == _cfg5_direct(gpu)
    assert "lost" in err and "requeued so far 0" not in err, err[-2000:]
