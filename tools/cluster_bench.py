"""Throughput of the server path against a direct search.

A client Request for "cmu440" over [0, 2^BITS) is served by mh_server with K
GPU miner threads on device 0.  Each thread loops over: take the next Request
written to it, run mh_miner_handle, and feed the Result back into the server.
This is the whole server + miner message path minus the LSP transport.  The
same range is also timed as one direct mh_search.  The ratio of the two is
the cost of chunking, JSON and scheduling.

    python tools/cluster_bench.py [--bits 36] [--miners 4] [--lose]

--lose drops one miner after its first chunk.  Its chunk is redone by the
others, and the answer must not change.
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]

import minehip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=36)
    ap.add_argument("--miners", type=int, default=4)
    ap.add_argument("--lose", action="store_true")
    ap.add_argument("--msg", default="cmu440")
    a = ap.parse_args()
    hi = (1 << a.bits) - 1
    minehip.search(a.msg, 0, 10 ** 6)  # warm up: context, code objects
    t0 = time.perf_counter()
    direct = minehip.search(a.msg, 0, hi)
    t_direct = time.perf_counter() - t0

    v = minehip.Server()
    miners = list(range(100, 100 + a.miners))
    inbox = {m: [] for m in miners}
    cv = threading.Condition()
    state = {"result": None, "lost": False, "chunks": 0}

    def now():
        return time.monotonic_ns()

    def route():  # caller holds cv
        for conn, payload in v.writes():
            if conn in inbox:
                inbox[conn].append(payload)
            else:
                state["result"] = json.loads(payload)
        cv.notify_all()

    def miner(m):
        while True:
            with cv:
                cv.wait_for(lambda: inbox[m] or state["result"] is not None)
                if state["result"] is not None:
                    return
                req = inbox[m].pop(0)
                if a.lose and not state["lost"] and m == miners[-1]:
                    state["lost"] = True
                    v.lost(m, now())
                    route()
                    return
            res = minehip.miner_handle(req)  # GPU; the GIL is released in ctypes
            with cv:
                v.read(m, res, now())
                state["chunks"] += 1
                route()

    t0 = time.perf_counter()
    with cv:
        for m in miners:
            v.read(m, minehip.marshal(minehip.NewJoin()), now())
        v.read(1, minehip.marshal(minehip.NewRequest(a.msg, 0, hi)), now())
        route()
    th = [threading.Thread(target=miner, args=(m,)) for m in miners]
    for t in th:
        t.start()
    for t in th:
        t.join()
    t_server = time.perf_counter() - t0
    r = state["result"]
    st = v.stats()
    out = {
        "range": f"[0, 2^{a.bits})", "msg": a.msg, "miners": a.miners, "lose_one": a.lose,
        "direct_ghs": round((hi + 1) / t_direct / 1e9, 3),
        "server_ghs": round((hi + 1) / t_server / 1e9, 3),
        "server_over_direct": round(t_direct / t_server, 4),
        "chunks": st["chunks_done"], "requeued": st["chunks_requeued"],
        "result": [r["Hash"], r["Nonce"]], "direct_result": list(direct),
        "match": [r["Hash"], r["Nonce"]] == list(direct),
    }
    print(json.dumps(out))
    return 0 if out["match"] else 1


if __name__ == "__main__":
    sys.exit(main())
