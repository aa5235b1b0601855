"""Throughput of the whole process layout of BASELINE configs[4] over LSP/UDP
on this box: bin/minehip-server, K bin/minehip-miner processes (GPU) and
bin/minehip-client, against one direct mh_search of the same range.

The client's wall time runs from its launch to its printed Result, so it
includes LSP connect, the Request, every chunk's Request/Result round trip,
JSON, scheduling and the final Result.  --kill SECONDS SIGKILLs one miner that
long after the client starts (dropped-miner recovery: detected by LSP epoch
timeout, LSP_EPOCH_MILLIS x LSP_EPOCH_LIMIT).

    python tools/lsp_cluster_bench.py [--bits 38] [--miners 1] [--gpus G] [--kill S]

--gpus G pins miner i to GPU i mod G (HIP_VISIBLE_DEVICES), one miner process per
GPU as in configs[4]: on an 8-GPU node, `--bits 42 --miners 8 --gpus 8 --kill 5`
is that config with a dropped miner.  --no-direct skips the direct-search
reference timing (which uses one GPU only).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitcoin-miner_amd")]
BIN = os.path.join(ROOT, "bitcoin-miner_amd", "bin")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bits", type=int, default=38)
    ap.add_argument("--miners", type=int, default=1)
    ap.add_argument("--kill", type=float, default=None)
    ap.add_argument("--msg", default="cmu440")
    ap.add_argument("--epoch-ms", type=int, default=200)
    ap.add_argument("--gpus", type=int, default=0, help="pin miner i to GPU i mod GPUS (0: no pinning)")
    ap.add_argument("--no-direct", action="store_true")
    a = ap.parse_args()
    hi = (1 << a.bits) - 1
    t_start = time.perf_counter()
    phase = ["start"]

    def heartbeat():  # a long run prints something every 30 s (gpurun treats silence as a hang)
        while True:
            time.sleep(30)
            print(f"[{time.perf_counter() - t_start:.0f} s] {phase[0]}", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()

    direct, t_direct = None, None
    if not a.no_direct:
        import minehip
        minehip.search(a.msg, 0, 10 ** 6)
        phase[0] = f"direct mh_search of 2^{a.bits}"
        t0 = time.perf_counter()
        direct = minehip.search(a.msg, 0, hi)
        t_direct = time.perf_counter() - t0

    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    hp = f"127.0.0.1:{port}"
    env = dict(os.environ, LSP_EPOCH_MILLIS=str(a.epoch_ms), LSP_EPOCH_LIMIT="5")
    procs = []
    try:
        srv = subprocess.Popen([os.path.join(BIN, "minehip-server"), str(port)], stdout=subprocess.PIPE,
                               stderr=subprocess.PIPE, env=env, text=True)
        procs.append(srv)
        srv.stdout.readline()
        miners = []
        for i in range(a.miners):
            menv = dict(env, HIP_VISIBLE_DEVICES=str(i % a.gpus)) if a.gpus else env
            miners.append(subprocess.Popen([os.path.join(BIN, "minehip-miner"), hp], stdout=subprocess.DEVNULL,
                                           stderr=subprocess.DEVNULL, env=menv))
        procs += miners
        time.sleep(3.0)  # miners joined and their GPU contexts up
        t0 = time.perf_counter()
        cl = subprocess.Popen([os.path.join(BIN, "minehip-client"), hp, a.msg, str(hi)], stdout=subprocess.PIPE,
                              env=env, text=True)
        procs.append(cl)
        phase[0] = f"LSP cluster, {a.miners} miner(s)"
        if a.kill is not None:
            time.sleep(a.kill)
            miners[-1].kill()
        out, _ = cl.communicate(timeout=3600)
        t_lsp = time.perf_counter() - t0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    err = srv.stderr.read()
    got = out.strip()
    n = hi + 1
    print(json.dumps({
        "msg": a.msg, "nonces": n, "miners": a.miners, "gpus": a.gpus or None, "killed_one_after_s": a.kill,
        "epoch_ms": a.epoch_ms,
        "direct": None if direct is None else {"s": round(t_direct, 3), "ghs": round(n / t_direct / 1e9, 3),
                                               "result": list(direct)},
        "lsp_cluster": {"s": round(t_lsp, 3), "ghs": round(n / t_lsp / 1e9, 3), "client_output": got},
        "ratio": None if direct is None else round(t_direct / t_lsp, 4),
        "match": None if direct is None else got == f"Result {direct[0]} {direct[1]}",
        "server_log": err.strip().splitlines()[-3:],
    }))


if __name__ == "__main__":
    main()
