"""CPU tests of the server side of the search (reference stub
bitcoin/server/server.go:62): the chunk scheduler (mh_sched_*) and the server
message loop (mh_server_*), include/minehip_server.h.

Miners are simulated here with the CPU oracle (test infrastructure) on small
ranges: the merged answer must equal the oracle's scan of the whole range,
whatever the chunking, miner speeds, losses and interleaving -- the
lexicographic min is associative, so anything else is a scheduler bug.  The
GPU form (miners = mh_miner_handle on the device) is in test_gpu_server.py.
"""
import json
import random
import threading

import pytest

import minehip
from minehip import Scheduler, Server, MinehipError
from oracle import oracle

U64 = (1 << 64) - 1


def covered(chunks):
    """Sorted, merged list of (lo, hi) from chunks; asserts no overlap."""
    out = []
    for lo, hi in sorted(chunks):
        if out:
            assert lo > out[-1][1], ("overlap", out[-1], (lo, hi))
            if lo == out[-1][1] + 1:
                out[-1] = (out[-1][0], hi)
                continue
        out.append((lo, hi))
    return out


def test_chunks_tile_the_range_in_order():
    s = Scheduler(init_chunk=100, min_chunk=100, max_chunk=100)
    s.add_miner(1)
    s.submit(9, "cmu440", 5, 1234)
    got = []
    while (a := s.next(now=0)) is not None:
        got.append((a[2], a[3]))
        r = s.result(1, 0, a[2], now=1)
    assert got[0] == (5, 104) and got[-1] == (1205, 1234)
    assert covered(got) == [(5, 1234)]
    assert r is not None and r[1] == 9  # completion for client 9
    st = s.stats()
    assert st["jobs"] == 0 and st["jobs_done"] == 1 and st["nonces_done"] == 1230


def test_top_of_u64_and_whole_u64_range():
    s = Scheduler(init_chunk=30, min_chunk=30, max_chunk=30)
    s.add_miner(0)
    s.submit(1, "x", U64 - 99, U64)
    chunks = []
    while (a := s.next(now=0)) is not None:
        chunks.append((a[2], a[3]))
        done = s.result(0, 5, a[3])
    assert covered(chunks) == [(U64 - 99, U64)] and len(chunks) == 4
    assert chunks[-1] == (U64 - 9, U64) and done == (0, 1, 5, U64 - 70)
    # the whole u64 range: 2^64 nonces, in 4 chunks of 2^62
    s = Scheduler(init_chunk=1 << 62, min_chunk=1 << 62, max_chunk=1 << 62)
    s.add_miner(0)
    s.submit(1, "x", 0, U64)
    chunks = []
    while (a := s.next(now=0)) is not None:
        chunks.append((a[2], a[3]))
        s.result(0, 5, a[2])
    assert chunks == [(k << 62, ((k + 1) << 62) - 1) for k in range(4)]


def test_result_merge_is_lexicographic_min():
    s = Scheduler(init_chunk=10, min_chunk=10, max_chunk=10)
    for m in (1, 2, 3):
        s.add_miner(m)
    s.submit(0, "m", 0, 29)
    a = [s.next(m, now=0) for m in (1, 2, 3)]
    assert [(x[2], x[3]) for x in a] == [(0, 9), (10, 19), (20, 29)]
    assert s.result(2, 7, 15) is None
    assert s.result(3, 7, 21) is None       # same hash, higher nonce: loses
    assert s.result(1, 8, 3) == (0, 0, 7, 15)


def test_round_robin_between_jobs():
    s = Scheduler(init_chunk=10, min_chunk=10, max_chunk=10)
    s.add_miner(1)
    ja = s.submit(100, "a", 0, 99)
    jb = s.submit(200, "b", 1000, 1019)
    order = []
    while (a := s.next(1, now=0)) is not None:
        order.append(a[1])
        s.result(1, 1, a[2])
    # alternate while both have work, then finish the long one
    assert order[:4] == [ja, jb, ja, jb] and order[4:] == [ja] * 8


def test_chunk_size_follows_rate_and_fair_share():
    s = Scheduler(init_chunk=1000, min_chunk=10, max_chunk=10 ** 9, target_ns=5000)
    s.add_miner(1)
    s.submit(0, "m", 0, 10 ** 6 - 1)
    a = s.next(1, now=0)
    assert a[3] - a[2] + 1 == 1000                   # init_chunk before any rate
    s.result(1, 1, a[2], now=1000)                   # 1 nonce/ns
    a = s.next(1, now=1000)
    assert a[3] - a[2] + 1 == 5000                   # rate x target
    s.result(1, 1, a[2], now=1000 + 2500)            # 2 nonces/ns -> EWMA 1.5
    a = s.next(1, now=3500)
    assert a[3] - a[2] + 1 == 7500
    # fair share: 2 miners, little work left -> at most pending / 4
    s2 = Scheduler(init_chunk=10 ** 6, min_chunk=1, max_chunk=10 ** 9)
    s2.add_miner(1)
    s2.add_miner(2)
    s2.submit(0, "m", 0, 999)
    a = s2.next(1)
    assert a[3] - a[2] + 1 == 1000 // 4
    b = s2.next(2)
    assert b[3] - b[2] + 1 == 750 // 4
    # a lone miner has no tail to share: its chunk is not halved
    s3 = Scheduler(init_chunk=10 ** 6, min_chunk=1, max_chunk=10 ** 9)
    s3.add_miner(1)
    s3.submit(0, "m", 0, 999)
    a = s3.next(1)
    assert (a[2], a[3]) == (0, 999)


def test_lost_miner_chunk_is_reassigned_first():
    s = Scheduler(init_chunk=10, min_chunk=10, max_chunk=10)
    s.add_miner(1)
    s.add_miner(2)
    s.submit(0, "m", 0, 49)
    a1 = s.next(1)
    a2 = s.next(2)
    s.remove_miner(1)
    assert s.stats()["chunks_requeued"] == 1
    s.result(2, 3, a2[2])
    assert s.next(2)[2:] == a1[2:]  # the lost chunk goes out before fresh work
    with pytest.raises(MinehipError):
        s.remove_miner(1)           # unknown now


def test_requeued_chunk_is_split_for_a_smaller_miner():
    s = Scheduler(init_chunk=100, min_chunk=1, max_chunk=100, target_ns=10)
    s.add_miner(1)
    s.add_miner(2)
    s.submit(0, "m", 0, 10 ** 6)
    assert s.next(1, now=0)[2:] == (0, 99)
    assert s.next(2, now=0)[2:] == (100, 199)
    s.remove_miner(1)                      # [0, 99] is requeued
    s.result(2, 1, 150, now=100)           # miner 2: 1 nonce/ns -> 10-nonce chunks
    assert s.next(2, now=100)[2:] == (0, 9)
    s.result(2, 1, 5, now=110)
    assert s.next(2, now=110)[2:] == (10, 19)


def test_out_of_chunk_nonce_is_rejected_and_requeued():
    s = Scheduler(init_chunk=10, min_chunk=10, max_chunk=10)
    s.add_miner(1)
    s.submit(0, "m", 0, 19)
    a = s.next(1)
    with pytest.raises(MinehipError) as e:
        s.result(1, 0, 15)  # nonce outside [0, 9]
    assert e.value.code == minehip.MH_ERANGE
    assert s.next(1)[2:] == a[2:]
    with pytest.raises(MinehipError):
        s.result(2, 0, 0)   # unknown miner / no chunk out


def test_client_drop_cancels_and_drains():
    s = Scheduler(init_chunk=10, min_chunk=10, max_chunk=10)
    s.add_miner(1)
    s.add_miner(2)
    s.submit(5, "m", 0, 99)
    keep = s.submit(6, "k", 0, 9)
    a1 = s.next(1)
    assert a1[1] == 0
    assert s.drop_client(5) == 1
    a2 = s.next(2)
    assert a2[1] == keep            # the cancelled job hands out nothing
    assert s.result(1, 1, a1[2]) is None   # late result of a cancelled job: ignored
    assert s.result(2, 4, 3) == (keep, 6, 4, 3)
    st = s.stats()
    assert st["jobs"] == 0 and st["jobs_cancelled"] == 1 and st["jobs_done"] == 1


def test_errors():
    with pytest.raises(MinehipError):
        Scheduler(min_chunk=10, max_chunk=5)
    s = Scheduler()
    with pytest.raises(MinehipError) as e:
        s.submit(0, "m", 5, 4)
    assert e.value.code == minehip.MH_ERANGE
    s.add_miner(3)
    with pytest.raises(MinehipError):
        s.add_miner(3)
    assert s.next(3) is None and s.next() is None
    assert s.job_msg(s.submit(0, b"\xffab", 0, 0)) == b"\xffab"


def simulate(seed, jobs, n_miners, p_loss=0.1, p_join=0.1, opts=None):
    """Event-driven simulation: miners with random speeds pick chunks, some
    are lost mid-chunk, new ones join; every chunk is scanned with the oracle.
    Returns {job id: (hash, nonce)} and the chunks completed per job."""
    rng = random.Random(seed)
    s = Scheduler(**(opts or dict(init_chunk=2000, min_chunk=300, max_chunk=20000, target_ns=10 ** 6)))
    ids = list(range(n_miners))
    for m in ids:
        s.add_miner(m)
    speed = {m: rng.uniform(0.2, 5.0) for m in ids}   # nonces per ns
    job_of = {}
    for k, (msg, lo, hi) in enumerate(jobs):
        job_of[s.submit(1000 + k, msg, lo, hi)] = (msg, lo, hi)
    now = 0
    busy = {}        # miner -> (finish time, assignment)
    done, chunks = {}, {j: [] for j in job_of}
    next_id = n_miners
    while len(done) < len(job_of):
        while (a := s.next(now=now)) is not None:
            m = a[0]
            busy[m] = (now + int((a[3] - a[2] + 1) / speed[m]) + 1, a)
        assert busy, "scheduler stalled with work left"
        m = min(busy, key=lambda x: busy[x][0])
        now, a = busy.pop(m)
        if rng.random() < p_loss and len(busy) + 1 > 1:
            s.remove_miner(m)           # lost mid-chunk: the work is redone elsewhere
        else:
            msg, _, _ = job_of[a[1]]
            h, n = oracle.search(msg, a[2], a[3], threads=1)
            chunks[a[1]].append((a[2], a[3]))
            r = s.result(m, h, n, now=now)
            if r is not None:
                done[r[0]] = (r[2], r[3])
        if rng.random() < p_join:
            s.add_miner(next_id)
            speed[next_id] = rng.uniform(0.2, 5.0)
            next_id += 1
    return done, chunks, job_of, s.stats()


def test_simulated_cluster_matches_oracle():
    jobs = [(b"cmu440", 0, 59_999), (b"x" * 60, 10 ** 9 - 7_000, 10 ** 9 + 20_000),
            (b"a" * 100, U64 - 25_000, U64), (b"", 123, 9_876)]
    done, chunks, job_of, st = simulate(440, jobs, n_miners=4)
    for j, (msg, lo, hi) in job_of.items():
        assert covered(chunks[j]) == [(lo, hi)]           # every nonce scanned exactly once
        assert done[j] == oracle.search(msg, lo, hi, threads=8), j
    assert st["jobs"] == 0 and st["chunks_requeued"] > 0  # losses happened and were recovered


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_simulated_cluster_seeds(seed):
    rng = random.Random(seed)
    jobs = []
    for _ in range(3):
        L = rng.randrange(0, 130)
        msg = bytes(rng.randrange(32, 127) for _ in range(L))
        lo = rng.choice([0, 10 ** rng.randrange(3, 19) - rng.randrange(0, 5000), U64 - 20_000])
        jobs.append((msg, lo, lo + rng.randrange(1, 20_000)))
    done, chunks, job_of, _ = simulate(seed, jobs, n_miners=rng.randrange(1, 6), p_loss=0.2)
    for j, (msg, lo, hi) in job_of.items():
        assert covered(chunks[j]) == [(lo, hi)]
        assert done[j] == oracle.search(msg, lo, hi, threads=8)


def test_concurrent_miner_threads():
    """Thread safety: miner threads pull chunks and post results concurrently."""
    s = Scheduler(init_chunk=500, min_chunk=500, max_chunk=500)
    msg, lo, hi = b"cmu440", 0, 39_999
    res = {}
    for m in range(6):
        s.add_miner(m)
    s.submit(1, msg, lo, hi)
    seen = []
    lock = threading.Lock()

    def run(m):
        while True:
            a = s.next(m)
            if a is None:
                if s.stats()["jobs"] == 0:
                    return
                continue
            h, n = oracle.search(msg, a[2], a[3], threads=1)
            with lock:
                seen.append((a[2], a[3]))
            r = s.result(m, h, n)
            if r is not None:
                res["r"] = (r[2], r[3])

    th = [threading.Thread(target=run, args=(m,)) for m in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert covered(seen) == [(lo, hi)]
    assert res["r"] == oracle.search(msg, lo, hi, threads=8)


# ---- the server message loop ---------------------------------------------

def J(payload):
    return json.loads(payload)


def test_server_join_request_result_flow():
    v = Server(init_chunk=1000, min_chunk=1000, max_chunk=1000)
    for miner in (10, 11):
        v.read(miner, minehip.marshal(minehip.NewJoin()))
    assert v.writes() == []
    v.read(1, minehip.marshal(minehip.NewRequest("cmu440", 0, 2_999)))   # client conn 1
    w = v.writes()
    assert [c for c, _ in w] == [10, 11]
    assert w[0][1] == b'{"Type":1,"Data":"cmu440","Lower":0,"Upper":999,"Hash":0,"Nonce":0}'
    assert J(w[1][1])["Lower"] == 1000 and J(w[1][1])["Upper"] == 1999
    # miner 10 answers; it gets the last chunk
    h, n = oracle.search("cmu440", 0, 999)
    v.read(10, minehip.marshal(minehip.NewResult(h, n)))
    w = v.writes()
    assert w == [(10, b'{"Type":1,"Data":"cmu440","Lower":2000,"Upper":2999,"Hash":0,"Nonce":0}')]
    for miner, (lo, hi) in ((11, (1000, 1999)), (10, (2000, 2999))):
        v.read(miner, minehip.marshal(minehip.NewResult(*oracle.search("cmu440", lo, hi))))
    exp = oracle.search("cmu440", 0, 2_999)
    assert v.writes() == [(1, minehip.marshal(minehip.NewResult(*exp)))]
    assert v.stats()["jobs_done"] == 1


def test_server_lost_miner_and_lost_client():
    v = Server(init_chunk=100, min_chunk=100, max_chunk=100)
    v.read(10, minehip.marshal(minehip.NewJoin()))
    v.read(11, minehip.marshal(minehip.NewJoin()))
    v.read(1, minehip.marshal(minehip.NewRequest("q", 0, 299)))
    w = v.writes()
    lost_chunk = J(w[0][1])
    v.lost(10, now=5)                 # miner 10 dies with [0, 99]
    assert v.writes() == []           # miner 11 still busy: nothing to hand out
    v.read(11, minehip.marshal(minehip.NewResult(*oracle.search("q", 100, 199))))
    w = v.writes()
    assert w[0][0] == 11 and (J(w[0][1])["Lower"], J(w[0][1])["Upper"]) == (lost_chunk["Lower"], lost_chunk["Upper"])
    # a second client, then the first client is lost: its job is dropped
    v.read(2, minehip.marshal(minehip.NewRequest("r", 5, 5)))
    v.lost(1)
    v.read(11, minehip.marshal(minehip.NewResult(*oracle.search("q", 0, 99))))
    w = v.writes()
    assert w == [(11, b'{"Type":1,"Data":"r","Lower":5,"Upper":5,"Hash":0,"Nonce":0}')]
    v.read(11, minehip.marshal(minehip.NewResult(oracle.hash_("r", 5), 5)))
    assert v.writes() == [(2, minehip.marshal(minehip.NewResult(oracle.hash_("r", 5), 5)))]
    st = v.stats()
    assert st["jobs_cancelled"] == 1 and st["jobs_done"] == 1 and st["jobs"] == 0


def test_server_rejects_bad_payloads():
    v = Server()
    with pytest.raises(MinehipError):
        v.read(1, b"not json")
    with pytest.raises(MinehipError):
        v.read(1, minehip.marshal(minehip.NewResult(1, 2)))  # no chunk out
    with pytest.raises(MinehipError):
        v.read(1, b'{"Type":7}')
    v.read(1, b'{"type":0}')                                  # Go: case-insensitive keys
    assert v.stats()["miners"] == 1


def test_server_refuses_unanswerable_requests():
    """A Request that can never get a Result (Lower > Upper, Data over MH_MAX_MSG_LEN) is refused
    with MH_EREJECTED and queues nothing: the transport then closes that client (minehip-server
    does; INTEGRATION.md's Go loop calls CloseConn), so it sees Disconnected instead of hanging."""
    v = Server()
    v.read(1, minehip.marshal(minehip.NewJoin()))
    with pytest.raises(MinehipError) as e:
        v.read(2, minehip.marshal(minehip.NewRequest("x", 9, 1)))
    assert e.value.code == minehip.MH_EREJECTED
    with pytest.raises(MinehipError) as e:
        v.read(3, minehip.marshal(minehip.NewRequest("y" * (minehip.MAX_MSG + 1), 0, 1)))
    assert e.value.code == minehip.MH_EREJECTED
    assert v.writes() == [] and v.stats()["jobs"] == 0
    v.lost(2)                                                  # the closed client: nothing to cancel
    v.read(4, minehip.marshal(minehip.NewRequest("z", 0, 9)))  # the server still works
    (c, payload), = v.writes()
    assert c == 1 and minehip.unmarshal(payload).Lower == 0


def test_server_writes_grow_for_escaped_data():
    """An encoded Request can be ~6x its Data (control bytes become \\u00XX): writes() grows its
    buffer to the reported size instead of failing on every later call."""
    v = Server()
    v.read(1, minehip.marshal(minehip.NewJoin()))
    data = "\x01" * 5000                                     # 30,000 bytes once escaped
    v.read(2, minehip.marshal(minehip.NewRequest(data, 0, 99)))
    (c, payload), = v.writes()
    m = minehip.unmarshal(payload)
    assert c == 1 and m.Data == data.encode() and len(payload) > 6 * 5000
    assert v.writes() == []
