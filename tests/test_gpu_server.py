"""GPU: the server loop (mh_server_*) driving GPU miners
(mh_miner_handle: Request payload -> Result payload on the device), with a
miner lost mid-job, against the oracle on small ranges and against a direct
mh_search at BASELINE's 2^32 size (plus the re-hash property).  Bit-exact."""
import json

import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

U64 = (1 << 64) - 1


def run_cluster(gpu, jobs, miners=(10, 11, 12), lose=None, **opts):
    """Serve `jobs` [(client, msg, lo, hi)] with GPU miners; `lose` = a miner
    that dies (without answering) after its first chunk.  Returns
    {client: (hash, nonce)} and the server's stats."""
    v = gpu.Server(**opts)
    for m in miners:
        v.read(m, gpu.marshal(gpu.NewJoin()))
    for c, msg, lo, hi in jobs:
        v.read(c, gpu.marshal(gpu.NewRequest(msg, lo, hi)))
    results, t = {}, 0
    pending = v.writes()
    lost = False
    while pending:
        conn, payload = pending.pop(0)
        t += 1
        if conn in miners:
            if conn == lose and not lost:
                lost = True
                v.lost(conn, now=t)           # dies holding this chunk
            else:
                v.read(conn, gpu.miner_handle(payload), now=t)
        else:
            m = json.loads(payload)
            assert m["Type"] == 2
            results[conn] = (m["Hash"], m["Nonce"])
        pending += v.writes()
    return results, v.stats()


def test_server_small_ranges_vs_oracle(gpu):
    jobs = [(1, b"cmu440", 0, 999_999), (2, b"x" * 60, 10 ** 9 - 5_000, 10 ** 9 + 300_000),
            (3, b"a" * 100, U64 - 200_000, U64), (4, b"", 7, 7)]
    res, st = run_cluster(gpu, jobs, lose=11, init_chunk=50_000, min_chunk=20_000, max_chunk=100_000)
    for c, msg, lo, hi in jobs:
        assert res[c] == oracle.search(msg, lo, hi, threads=8), c
    assert st["chunks_requeued"] == 1 and st["jobs_done"] == 4 and st["jobs"] == 0


def test_server_config2_size(gpu):
    """BASELINE configs[1] range through the server, one miner lost."""
    hi = (1 << 32) - 1
    exp = gpu.search("cmu440", 0, hi)
    res, st = run_cluster(gpu, [(1, "cmu440", 0, hi)], lose=12, init_chunk=1 << 28)
    assert res[1] == exp
    assert oracle.hash_("cmu440", exp[1]) == exp[0]
    assert st["chunks_requeued"] == 1


def test_search_multi_adaptive_and_fixed(gpu):
    hi = (1 << 32) - 1
    exp = gpu.search("cmu440", 0, hi)
    assert gpu.search_multi("cmu440", 0, hi, devs=[0, 0, 0, 0]) == exp       # adaptive chunks
    assert gpu.search_multi("cmu440", 0, hi, devs=[0, 0], chunk=(1 << 26) + 17) == exp


def test_search_multi_rates_persist(gpu):
    """Adaptive search_multi measures each device's rate on its shard (>= 2^30 nonces) and keeps
    it for the next call's split; the answer does not depend on the split."""
    hi = (1 << 33) - 1
    exp = gpu.search("cmu440", 0, hi)
    assert gpu.search_multi("cmu440", 0, hi, devs=[0, 0]) == exp
    r = gpu.multi_rates([0])[0]
    assert r > 0.0
    # slots per ns: one MI355X issues ~1e5 (nonce_cost slots ~2,000 x ~50 nonces/ns)
    assert 1e4 < r < 1e6, r
    assert gpu.search_multi("cmu440", 0, hi, devs=[0, 0, 0]) == exp


def test_search_multi_device_failure_hand_back(gpu):
    """A worker whose device fails hands its chunk (fixed chunks) or its whole shard (adaptive,
    split over the workers still running) back; the others finish with the same answer.  If every
    worker fails, the call fails.  The failure is injected by the dev build's
    MINEHIP_TEST_FAIL_WORKER hook, in a child process (the product library has no hooks)."""
    from conftest import run_dev
    hi = (1 << 31) - 1
    exp = gpu.search("cmu440", 0, hi)
    r = run_dev(f"""
import os, minehip
os.environ["MINEHIP_TEST_FAIL_WORKER"] = "1"
print(*minehip.search_multi("cmu440", 0, {hi}, devs=[0, 0, 0], chunk=1 << 27))
print(*minehip.search_multi("cmu440", 0, {hi}, devs=[0, 0, 0]))
os.environ["MINEHIP_TEST_FAIL_WORKER"] = "0"   # the only worker fails
for chunk in (1 << 27, 0):
    try:
        minehip.search_multi("cmu440", 0, {hi}, devs=[0], chunk=chunk)
        raise SystemExit("search_multi succeeded with its only worker failing")
    except minehip.MinehipError as e:
        assert e.code == minehip.MH_EHIP and "injected" in str(e), e
""")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()[-2:]
    assert [tuple(int(x) for x in ln.split()) for ln in lines] == [exp, exp]


def test_search_multi_thread_start_failure(gpu):
    """Host threads that cannot start: with the dev build's MINEHIP_TEST_SPAWN_LIMIT=k
    only the first k workers' threads start.  k > 0: the started workers take the others' shards
    (adaptive) or chunks (fixed) and the answer is unchanged; k = 0: MH_EINTERNAL, nothing searched."""
    from conftest import run_dev
    hi = (1 << 31) - 1
    exp = gpu.search("cmu440", 0, hi)
    r = run_dev(f"""
import os, minehip
os.environ["MINEHIP_TEST_SPAWN_LIMIT"] = "1"
print(*minehip.search_multi("cmu440", 0, {hi}, devs=[0, 0, 0], chunk=1 << 27))
print(*minehip.search_multi("cmu440", 0, {hi}, devs=[0, 0, 0]))
os.environ["MINEHIP_TEST_SPAWN_LIMIT"] = "0"
for chunk in (1 << 27, 0):
    try:
        minehip.search_multi("cmu440", 0, {hi}, devs=[0, 0], chunk=chunk)
        raise SystemExit("search_multi succeeded with no worker thread started")
    except minehip.MinehipError as e:
        assert e.code == minehip.MH_EINTERNAL and "could not start" in str(e), e
""")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()[-2:]
    assert [tuple(int(x) for x in ln.split()) for ln in lines] == [exp, exp]
