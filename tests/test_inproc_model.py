"""tools/inproc_model.py (the one-GPU model of the in-process N-GPU path) on CPU: the replayed
round-3 scheduler chain and the round-4 shards each cover the step once and merge to the whole
range's answer.  The searches are the oracle here; on the box they are minehip.search."""
import os
import sys
import types

import minehip
from conftest import ROOT
from oracle import oracle

sys.path.insert(0, os.path.join(ROOT, "tools"))
import inproc_model  # noqa: E402


def fake_minehip(calls):
    m = types.SimpleNamespace()

    def search(msg, lo, hi):
        calls.append((lo, hi))
        return oracle.search(msg, lo, hi)

    m.search = search
    m.Scheduler = minehip.Scheduler
    m.multi_plan = minehip.multi_plan
    return m


def tiles(calls, lo, hi):
    rs = sorted(calls)
    return rs[0][0] == lo and rs[-1][1] == hi and all(a[1] + 1 == b[0] for a, b in zip(rs, rs[1:]))


def test_old_and_new_paths_cover_the_step_once():
    msg, lo, hi = b"cmu440", 0, (1 << 17) - 1
    exp = list(oracle.search(msg, lo, hi))
    for n in (2, 4, 8):
        calls = []
        old = inproc_model.old_path(fake_minehip(calls), msg, lo, hi, n)
        assert old["result"] == exp and old["merged"] == exp
        assert tiles(calls, lo, hi) and sum(old["chunks_per_device"]) == len(calls)
        assert old["step_ms"] > 0
        calls = []
        new = inproc_model.new_path(fake_minehip(calls), msg, lo, hi, n)
        assert new["result"] == exp and tiles(calls, lo, hi)
        assert len(calls) == new["spans"] <= n  # one shard per device at this size (no tail)
