"""End-to-end rehearsal of BASELINE configs[4]: a server, several miner
processes and a client, in separate processes, with dropped-miner recovery.

This is the reference's process layout (bitcoin/server, bitcoin/miner,
bitcoin/client).  The LSP transport (lsp/, lspnet/) is Go
and stays the reference's.  This harness stands in for it with the simplest
reliable framing: TCP on 127.0.0.1, each message a 4-byte big-endian length
followed by the payload.  The payloads are exactly what travels over LSP, Go
encoding/json bitcoin.Messages.  The server runs the library's server loop
(mh_server_*).  A GPU miner runs mh_miner_handle on its device.

    python tools/cluster.py server PORT [--chunk N]
    python tools/cluster.py miner  HOST:PORT [--dev D] [--drop-after N]
    python tools/cluster.py client HOST:PORT MESSAGE MAXNONCE

The client prints "Result <hash> <nonce>" or "Disconnected", as
bitcoin/client/client.go:41-48 does.  tests/e2e_oracle_miner.py is a CPU
miner built from the test oracle on the same framing, so that
tests/test_e2e_cluster.py can run this harness on a host without a GPU.
"""
import argparse
import os
import queue
import socket
import struct
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]

import minehip  # noqa: E402


def send_msg(sock, payload):
    sock.sendall(struct.pack(">I", len(payload)) + payload)


def recv_exact(sock, n):
    buf = b""
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("closed")
        buf += chunk
    return buf


def recv_msg(sock):
    (n,) = struct.unpack(">I", recv_exact(sock, 4))
    return recv_exact(sock, n)


def connect(hostport, tries=100):
    host, port = hostport.rsplit(":", 1)
    for i in range(tries):
        try:
            return socket.create_connection((host, int(port)))
        except OSError:
            time.sleep(0.1)
    raise ConnectionError(f"cannot connect to {hostport}")


def server(port, chunk):
    """bitcoin/server: events from every connection go through one loop that
    drives mh_server (server.go:62 TODO)."""
    opts = {} if not chunk else dict(init_chunk=chunk, min_chunk=chunk, max_chunk=chunk)
    v = minehip.Server(**opts)
    events = queue.Queue()
    conns = {}
    lock = threading.Lock()
    ls = socket.socket()
    ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    ls.bind(("127.0.0.1", port))
    ls.listen(64)
    print(f"Server listening on port {port}", flush=True)

    def reader(cid, s):
        try:
            while True:
                events.put((cid, recv_msg(s)))
        except (ConnectionError, OSError):
            events.put((cid, None))  # lost, like lsp.Server.Read's error return

    def acceptor():
        cid = 0
        while True:
            s, _ = ls.accept()
            cid += 1
            with lock:
                conns[cid] = s
            threading.Thread(target=reader, args=(cid, s), daemon=True).start()

    threading.Thread(target=acceptor, daemon=True).start()
    t0 = time.monotonic_ns()
    while True:
        cid, payload = events.get()
        now = time.monotonic_ns() - t0
        try:
            if payload is None:
                with lock:
                    conns.pop(cid, None)
                v.lost(cid, now)
            else:
                v.read(cid, payload, now)
        except minehip.MinehipError as e:
            print(f"conn {cid}: {e}", file=sys.stderr, flush=True)
        for c, p in v.writes():
            with lock:
                s = conns.get(c)
            if s is not None:
                try:
                    send_msg(s, p)
                except OSError:
                    pass  # its reader reports the loss


def miner(hostport, dev, handle=None, drop_after=0):
    """bitcoin/miner: Join, then Request -> search -> Result until the server
    goes away.  drop_after=N: vanish on receiving the N-th chunk, without
    answering (a miner lost mid-chunk, for the recovery tests)."""
    s = connect(hostport)
    send_msg(s, minehip.marshal(minehip.NewJoin()))
    if handle is None:
        def handle(p):
            return minehip.miner_handle(p, devs=(dev,))
    print("miner joined", flush=True)
    n = 0
    try:
        while True:
            req = recv_msg(s)
            n += 1
            if n == drop_after:
                print("dropping", flush=True)
                s.close()
                return
            send_msg(s, handle(req))
    except (ConnectionError, OSError):
        return


def client(hostport, message, max_nonce):
    """bitcoin/client (client.go:25-48): one Request [0, maxNonce], print the Result."""
    s = connect(hostport)
    send_msg(s, minehip.marshal(minehip.NewRequest(message, 0, max_nonce)))
    try:
        m = minehip.unmarshal(recv_msg(s))
        print("Result", m.Hash, m.Nonce, flush=True)
    except (ConnectionError, OSError):
        print("Disconnected", flush=True)


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("server")
    a.add_argument("port", type=int)
    a.add_argument("--chunk", type=int, default=0)
    a = sub.add_parser("miner")
    a.add_argument("hostport")
    a.add_argument("--dev", type=int, default=0)
    a.add_argument("--drop-after", type=int, default=0)
    a = sub.add_parser("client")
    a.add_argument("hostport")
    a.add_argument("message")
    a.add_argument("max_nonce", type=int)
    args = ap.parse_args()
    if args.cmd == "server":
        server(args.port, args.chunk)
    elif args.cmd == "miner":
        miner(args.hostport, args.dev, drop_after=args.drop_after)
    else:
        client(args.hostport, args.message, args.max_nonce)


if __name__ == "__main__":
    main()
