"""CPU tests of liblsp440 (include/lsp440.h), the LSP endpoint the native
miner / server / client processes use.

Two kinds of test:
  * restatements of the reference's own LSP test suites (lsp/lsp1_test.go
    basic echo + robustness under packet loss, lsp2_test.go windows,
    lsp3_test.go epochs / lost peers, lsp4_test.go close, lsp5_test.go
    variable-length messages), with lspnet's fault injection replaced by
    lsp_set_drop_percent / lsp_set_msg_mangle_percent;
  * wire tests against a raw UDP peer written here from lsp/message.go and
    lsp/util.go: exact datagram bytes (Go encoding/json of lsp.Message), the
    sliding window, epoch resends and heartbeats, out-of-order delivery.
    They pin wire compatibility with the reference's Go endpoints, which
    cannot run here (no Go toolchain).
"""
import base64
import json
import os
import random
import re
import socket
import threading
import time

import pytest

from conftest import ROOT
from minehip import lsp


@pytest.fixture(autouse=True)
def clean_faults():
    lsp.set_drop_percent(0, 0, 0, 0)
    lsp.set_msg_mangle_percent(0, 0)
    yield
    lsp.set_drop_percent(0, 0, 0, 0)
    lsp.set_msg_mangle_percent(0, 0)


def test_exports_every_declared_symbol():
    import ctypes
    src = open(os.path.join(ROOT, "include", "lsp440.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    syms = set(re.findall(r"\b(lsp_[a-z_0-9]+)\s*\(", src))
    assert syms == set(lsp.EXPORTS)
    raw = ctypes.CDLL(lsp.LIB_PATH)
    for s in syms:
        assert hasattr(raw, s), s


# ---- wire format (lsp/message.go:17-24, lsp/util.go:19-33) -------------------

def test_marshal_is_go_json():
    # json.Marshal(&Message{...}): fields in declaration order, []byte as
    # base64 (StdEncoding, padded), nil slice as null.
    assert lsp.marshal(lsp.MsgConnect) == b'{"Type":0,"ConnID":0,"SeqNum":0,"Size":0,"Payload":null}'
    assert lsp.marshal(lsp.MsgData, 3, 7, 5, b"hello") == \
        b'{"Type":1,"ConnID":3,"SeqNum":7,"Size":5,"Payload":"aGVsbG8="}'
    assert lsp.marshal(lsp.MsgAck, 3, 7) == b'{"Type":2,"ConnID":3,"SeqNum":7,"Size":0,"Payload":null}'
    assert lsp.marshal(lsp.MsgData, 1, 1, 0, b"") == b'{"Type":1,"ConnID":1,"SeqNum":1,"Size":0,"Payload":""}'
    rng = random.Random(440)
    for n in list(range(0, 10)) + [255, 256, 999]:
        p = bytes(rng.randrange(256) for _ in range(n))
        got = json.loads(lsp.marshal(lsp.MsgData, 9, 2, n, p))
        assert got == {"Type": 1, "ConnID": 9, "SeqNum": 2, "Size": n, "Payload": base64.b64encode(p).decode()}


def test_unmarshal_follows_go_rules():
    # case-insensitive keys, unknown keys ignored, missing fields zero, whitespace
    m = lsp.unmarshal(b' { "type" : 1, "CONNID":4, "seqnum":2, "size":3, "Payload":"YWJj", "x":[1,{"y":null}] } ')
    assert m == {"Type": 1, "ConnID": 4, "SeqNum": 2, "Size": 3, "Payload": b"abc"}
    assert lsp.unmarshal(b'{"Type":2}') == {"Type": 2, "ConnID": 0, "SeqNum": 0, "Size": 0, "Payload": None}
    for bad in (b"", b"[]", b'{"Type":1', b'{"Payload":"abc"}', b'{"Type":"1"}', b'{"Type":1.5}',
                b'{"Type":1} x'):
        assert lsp.unmarshal(bad) is None, bad
    for p in (b"", b"a", b"ab", b"abc", bytes(range(256))):
        assert lsp.unmarshal(lsp.marshal(1, 1, 1, len(p), p))["Payload"] == p


# ---- helpers ------------------------------------------------------------------

def fast(limit=5, millis=100, window=1):
    return lsp.Params(limit, millis, window)


class Echo:
    """An LSP echo server in a thread (lsp1_test.go's server side)."""

    def __init__(self, params):
        self.srv, err = lsp.NewServer(0, params)
        assert err is None
        self.events = []
        self.t = threading.Thread(target=self.run, daemon=True)
        self.t.start()

    @property
    def hostport(self):
        return f"localhost:{self.srv.port}"

    def run(self):
        while True:
            c, p, err = self.srv.Read()
            if err is not None:
                self.events.append((c, err.code))
                if c == 0:
                    return
                continue
            self.srv.Write(c, p)

    def close(self):
        r = self.srv.Close()
        self.t.join(10)
        return r


def echo_round(params, n_clients, n_msgs, timeout=60):
    e = Echo(params)
    clients = []
    for _ in range(n_clients):
        c, err = lsp.NewClient(e.hostport, params)
        assert err is None, err
        clients.append(c)
    assert len({c.ConnID() for c in clients}) == n_clients
    fails = []

    def one(c, k):
        msgs = [f"{k}:{i}:{random.getrandbits(64)}".encode() for i in range(n_msgs)]
        for m in msgs:
            assert c.Write(m) is None
        for m in msgs:
            got, err = c.Read(timeout_ms=timeout * 1000)
            if err is not None or got != m:
                fails.append((k, m, got, err))
                return

    ts = [threading.Thread(target=one, args=(c, k)) for k, c in enumerate(clients)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
    lsp.set_drop_percent(0, 0, 0, 0)
    lsp.set_msg_mangle_percent(0, 0)
    for c in clients:
        assert c.Close() is None
    e.close()
    assert not fails, fails[:3]


# ---- lsp1_test.go: basic echo and robustness -----------------------------------

@pytest.mark.parametrize("n_clients,n_msgs,window", [(1, 1, 1), (1, 100, 1), (3, 50, 1), (5, 100, 5),
                                                     (10, 30, 10)])
def test_basic_echo(n_clients, n_msgs, window):
    echo_round(fast(window=window), n_clients, n_msgs)


@pytest.mark.parametrize("n_clients,n_msgs,window", [(1, 20, 1), (3, 20, 4)])
def test_robust_echo_with_packet_loss(n_clients, n_msgs, window):
    # TestRobust*: 20% of datagrams dropped in every direction; every message
    # still arrives exactly once and in order (epoch resends).
    lsp.set_drop_percent(20, 20, 20, 20)
    echo_round(fast(limit=20, millis=20, window=window), n_clients, n_msgs)


# ---- lsp5_test.go: variable-length messages --------------------------------------

def test_shortened_and_lengthened_payloads():
    # A Data whose payload is shorter than Size is dropped (and later resent),
    # a longer one is truncated to Size.
    lsp.set_msg_mangle_percent(30, 30)
    echo_round(fast(limit=20, millis=20, window=2), 2, 30)


# ---- raw UDP peer: exact wire behaviour ----------------------------------------

class RawPeer:
    """A bare UDP socket speaking the reference's datagrams (lsp/message.go)."""

    def __init__(self):
        self.s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.s.bind(("127.0.0.1", 0))
        self.port = self.s.getsockname()[1]
        self.addr = None

    def recv(self, timeout=1.0):
        self.s.settimeout(timeout)
        try:
            b, self.addr = self.s.recvfrom(65536)
        except socket.timeout:
            return None, None
        return json.loads(b), b

    def drain(self, seconds):
        out, end = [], time.time() + seconds
        while time.time() < end:
            m, _ = self.recv(max(0.01, end - time.time()))
            if m is not None:
                out.append(m)
        return out

    def send(self, type_, conn=0, seq=0, payload=None, size=None):
        size = len(payload) if size is None and payload is not None else (size or 0)
        self.s.sendto(lsp.marshal(type_, conn, seq, size, payload), self.addr)

    def close(self):
        self.s.close()


def connect_raw(params, conn_id=7):
    peer = RawPeer()
    box = {}
    t = threading.Thread(target=lambda: box.update(r=lsp.NewClient(f"127.0.0.1:{peer.port}", params)))
    t.start()
    m, raw = peer.recv(5)
    assert raw == b'{"Type":0,"ConnID":0,"SeqNum":0,"Size":0,"Payload":null}'
    peer.send(lsp.MsgAck, conn_id, 0)
    t.join(5)
    cl, err = box["r"]
    assert err is None and cl.ConnID() == conn_id
    return peer, cl


def test_client_window_and_epoch_resend():
    # lsp2_test.go (windows): with WindowSize W only seq < oldest unacked + W
    # may be in flight; unacked ones are resent every epoch.
    peer, cl = connect_raw(fast(limit=50, millis=100, window=3))
    for i in range(1, 9):
        assert cl.Write(f"m{i}".encode()) is None
    seen = [m for m in peer.drain(0.45) if m["Type"] == lsp.MsgData]
    seqs = {m["SeqNum"] for m in seen}
    assert seqs == {1, 2, 3}, seqs
    assert sum(m["SeqNum"] == 1 for m in seen) >= 3  # first send + epoch resends
    m1 = next(m for m in seen if m["SeqNum"] == 1)
    assert m1 == {"Type": 1, "ConnID": 7, "SeqNum": 1, "Size": 2, "Payload": base64.b64encode(b"m1").decode()}
    peer.send(lsp.MsgAck, 7, 2)  # out of order: the window still starts at 1
    seqs = {m["SeqNum"] for m in peer.drain(0.25) if m["Type"] == lsp.MsgData}
    assert seqs <= {1, 3}, seqs
    peer.send(lsp.MsgAck, 7, 1)  # now 1, 2 acked: 3, 4, 5 may fly
    seqs = {m["SeqNum"] for m in peer.drain(0.25) if m["Type"] == lsp.MsgData}
    assert seqs == {3, 4, 5}, seqs
    for s in range(3, 9):
        peer.send(lsp.MsgAck, 7, s)
    assert cl.Close() is None  # everything acked: Close returns
    peer.close()


def test_client_delivers_in_order_once_and_acks():
    peer, cl = connect_raw(fast(limit=50, millis=200, window=4))
    peer.send(lsp.MsgData, 7, 2, b"two")
    peer.send(lsp.MsgData, 7, 1, b"one")
    peer.send(lsp.MsgData, 7, 1, b"one")      # duplicate: acked, not delivered again
    peer.send(lsp.MsgData, 7, 3, b"thr", size=5)  # shorter than Size: dropped, not acked
    peer.send(lsp.MsgData, 7, 3, b"three!!", size=5)  # longer: truncated to Size
    assert cl.Read(2000) == (b"one", None)
    assert cl.Read(2000) == (b"two", None)
    assert cl.Read(2000) == (b"three", None)
    assert cl.Read(300)[1].code == lsp.LSP_ETIMEOUT
    acks = [m["SeqNum"] for m in peer.drain(0.1) if m["Type"] == lsp.MsgAck]
    assert sorted(set(acks)) == [1, 2, 3] and acks.count(1) >= 2
    cl.Close()
    peer.close()


def test_client_heartbeat_then_lost():
    # lsp3_test.go: no Data yet -> Ack(connID, 0) every epoch; a silent server
    # is lost after EpochLimit epochs and Read then fails.
    limit, millis = 4, 100
    peer, cl = connect_raw(fast(limit=limit, millis=millis, window=1))
    t0 = time.time()
    hb = [m for m in peer.drain(0.35) if m["Type"] == lsp.MsgAck]
    assert len(hb) >= 2 and all(m["SeqNum"] == 0 and m["ConnID"] == 7 for m in hb)
    got, err = cl.Read(5000)
    dt = time.time() - t0
    assert got is None and err.code == lsp.LSP_ELOST
    # lost no earlier than EpochLimit epochs; the upper bound leaves room for a loaded host
    # (the CPU suite may run beside multi-threaded oracle scans)
    assert limit * millis / 1e3 <= dt <= (limit + 3) * millis / 1e3 + 1.0, dt
    assert cl.Read(100)[1].code == lsp.LSP_ELOST  # sticky
    assert cl.Write(b"x").code == lsp.LSP_ELOST
    cl.Close()
    peer.close()


def test_connect_fails_after_epoch_limit():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))  # bound but silent: Connects go unanswered
    port = s.getsockname()[1]
    t0 = time.time()
    cl, err = lsp.NewClient(f"127.0.0.1:{port}", fast(limit=3, millis=50))
    assert cl is None and err.code == lsp.LSP_ECONNECT
    assert 0.15 <= time.time() - t0 < 2.0
    connects = 0
    s.settimeout(0.05)
    try:
        while True:
            connects += json.loads(s.recv(1000))["Type"] == lsp.MsgConnect
    except socket.timeout:
        pass
    assert connects >= 3  # the first Connect + one per epoch
    s.close()


def test_server_acks_connect_once_per_address():
    srv, _ = lsp.NewServer(0, fast(limit=50, millis=100))
    peer = RawPeer()
    peer.addr = ("127.0.0.1", srv.port)
    peer.send(lsp.MsgConnect)
    m, _ = peer.recv(2)
    assert m["Type"] == lsp.MsgAck and m["SeqNum"] == 0 and m["ConnID"] >= 1
    cid = m["ConnID"]
    peer.send(lsp.MsgConnect)  # resent Connect (our Ack "lost"): same connID
    m2 = next(x for x in peer.drain(0.3) if x["Type"] == lsp.MsgAck)
    assert m2["ConnID"] == cid
    peer.send(lsp.MsgData, cid, 1, b"hi")
    assert srv.Read(2000) == (cid, b"hi", None)
    peer.send(lsp.MsgData, cid + 100, 1, b"nobody")  # unknown connID: ignored
    assert srv.Read(300)[2].code == lsp.LSP_ETIMEOUT
    assert srv.Write(cid + 100, b"x").code == lsp.LSP_EINVAL
    peer.close()
    srv.Close()


# ---- lost connections and close (lsp4_test.go) ---------------

def test_server_read_reports_lost_client_after_its_messages():
    # server_api.go:7-17: Read returns (connID, err) for a lost client once no
    # message of it is waiting.  The reference server never does (N3).
    p = fast(limit=3, millis=50)
    srv, _ = lsp.NewServer(0, p)
    cl, _ = lsp.NewClient(f"127.0.0.1:{srv.port}", p)
    cid = cl.ConnID()
    for m in (b"a", b"b", b"c"):
        cl.Write(m)
    assert cl.Close() is None  # returns once all three are acked; then the client is silent
    assert [srv.Read(2000)[1] for _ in range(3)] == [b"a", b"b", b"c"]
    c, got, err = srv.Read(3000)
    assert (c, got, err.code) == (cid, None, lsp.LSP_ELOST)
    # the report freed the connection's state; its id still answers "lost"
    assert srv.Write(cid, b"late").code == lsp.LSP_ELOST
    assert srv.CloseConn(cid).code == lsp.LSP_ECLOSED
    srv.Close()


def test_oversized_write_fails_instead_of_hanging():
    # a Data frame larger than one UDP datagram could never be delivered: the
    # write is refused (LSP_ETOOBIG) and the connection stays usable
    p = fast(limit=20, millis=50)
    srv, _ = lsp.NewServer(0, p)
    cl, _ = lsp.NewClient(f"127.0.0.1:{srv.port}", p)
    big = b"\x00" * lsp.MAX_DATAGRAM  # base64 grows it by 4/3
    assert cl.Write(big).code == lsp.LSP_ETOOBIG
    assert cl.Write(b"\x00" * 40000) is None  # 53 KB frame: still one datagram
    c, got, err = srv.Read(3000)
    assert err is None and got == b"\x00" * 40000
    assert srv.Write(c, big).code == lsp.LSP_ETOOBIG
    assert srv.Write(c, b"ok") is None
    assert cl.Read(3000) == (b"ok", None)
    assert cl.Close() is None
    srv.Close()


def test_close_conn_and_server_close():
    p = fast(limit=10, millis=50)
    srv, _ = lsp.NewServer(0, p)
    a, _ = lsp.NewClient(f"127.0.0.1:{srv.port}", p)
    b, _ = lsp.NewClient(f"127.0.0.1:{srv.port}", p)
    assert srv.Write(a.ConnID(), b"bye") is None
    assert srv.CloseConn(a.ConnID()) is None  # non-blocking; "bye" still delivered
    assert a.Read(2000) == (b"bye", None)
    c, got, err = srv.Read(2000)
    assert c == a.ConnID() and err.code == lsp.LSP_ECLOSED
    assert srv.Write(a.ConnID(), b"x") is not None
    box = {}
    reader = threading.Thread(target=lambda: box.update(r=srv.Read()))
    reader.start()
    time.sleep(0.1)
    srv.Write(b.ConnID(), b"last")
    assert srv.Close() is None  # blocks until "last" is acked
    reader.join(5)
    assert box["r"][0] == 0 and box["r"][2].code == lsp.LSP_ECLOSED
    assert b.Read(2000) == (b"last", None)
    a.Close()
    b.Close()


def test_server_close_reports_a_conn_lost_while_closing_after_read_reported_it():
    """a connection lost during CloseConn with data still unacked makes Server.Close
    return LSP_ELOST -- also when Read has already reported the loss and freed the connection."""
    p = fast(limit=3, millis=50)
    srv, _ = lsp.NewServer(0, p)
    peer = RawPeer()
    peer.addr = ("127.0.0.1", srv.port)
    peer.send(lsp.MsgConnect)
    m, _ = peer.recv(2)
    cid = m["ConnID"]
    peer.close()                                  # the client goes silent: nothing is ever acked
    assert srv.Write(cid, b"never acked") is None
    assert srv.CloseConn(cid) is None
    c, got, err = srv.Read(3000)                  # lost while closing, reported, then forgotten
    assert (c, got, err.code) == (cid, None, lsp.LSP_ELOST)
    assert srv.Write(cid, b"x").code == lsp.LSP_ELOST
    err = srv.Close()
    assert err is not None and err.code == lsp.LSP_ELOST


def test_client_close_waits_for_acks_under_loss():
    # lsp4_test.go ClientClose: Close blocks until pending messages are acked,
    # here with the network dropping everything at first.
    p = fast(limit=40, millis=30, window=2)
    e = Echo(p)
    cl, _ = lsp.NewClient(e.hostport, p)
    lsp.set_drop_percent(0, 100, 0, 0)
    for i in range(5):
        cl.Write(b"%d" % i)
    threading.Timer(0.3, lambda: lsp.set_drop_percent(0, 0, 0, 0)).start()
    t0 = time.time()
    assert cl.Close() is None
    assert time.time() - t0 >= 0.2
    time.sleep(0.1)
    e.close()


def test_server_slow_start():
    # lsp3_test.go TestServerSlowStart: the client dials before the server is
    # up; its Connect is resent every epoch until the server answers.
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()  # a free port, nobody listening yet
    p = fast(limit=20, millis=50)
    box = {}
    t = threading.Thread(target=lambda: box.update(r=lsp.NewClient(f"127.0.0.1:{port}", p)))
    t.start()
    time.sleep(0.3)
    srv, err = lsp.NewServer(port, p)
    assert err is None
    t.join(5)
    cl, err = box["r"]
    assert err is None and cl.ConnID() >= 1
    assert cl.Write(b"late") is None
    assert srv.Read(2000) == (cl.ConnID(), b"late", None)
    cl.Close()
    srv.Close()


def test_every_client_ticks_independently():
    # The reference server shares one time.Ticker among its per-client
    # goroutines (lsp/server_impl.go:47,137), so each tick reaches one client
    # and a loss stops it for all.  Here every connection is
    # checked every epoch: two silent clients are both reported lost, and a
    # third, live one is not.  (5 x 100 ms: a live client's heartbeat thread must not look
    # silent on a loaded host, where 3 x 50 ms was once too tight under pytest -n.)
    p = fast(limit=5, millis=100)
    srv, _ = lsp.NewServer(0, p)
    a, _ = lsp.NewClient(f"127.0.0.1:{srv.port}", p)
    b, _ = lsp.NewClient(f"127.0.0.1:{srv.port}", p)
    live, _ = lsp.NewClient(f"127.0.0.1:{srv.port}", p)
    ids = {a.ConnID(), b.ConnID()}
    a.Close()
    b.Close()
    lost = set()
    t0 = time.time()
    while len(lost) < 2 and time.time() - t0 < 3:
        c, _, err = srv.Read(3000)
        assert err is not None and err.code == lsp.LSP_ELOST
        lost.add(c)
    assert lost == ids
    assert srv.Read(400)[2].code == lsp.LSP_ETIMEOUT  # the live client keeps heartbeating
    assert live.Write(b"still here") is None
    assert srv.Read(2000) == (live.ConnID(), b"still here", None)
    live.Close()
    srv.Close()
