"""Native C++ front ends of the C-ABI (bitcoin-miner_amd/csrc/cli.cpp,
csrc/apps/miner_main.cpp).

minehip-search mirrors the reference client's arguments and output
(bitcoin/client/client.go:12-19, :41-43); `minehip-miner --stdio` is the
miner's Request -> Result step over JSON lines (bitcoin/message.go:27-44).
The processes over LSP are tested in test_e2e_cluster.py."""
import os
import subprocess

import pytest

from conftest import PKG

BIN = os.path.join(PKG, "bin")


def run(name, *args, stdin=None):
    return subprocess.run([os.path.join(BIN, name), *args], input=stdin, capture_output=True, text=True,
                          timeout=300)


def test_usage_and_number_errors():
    r = run("minehip-search", "cmu440")
    assert r.returncode == 2 and r.stdout.startswith("Usage: ")
    r = run("minehip-search", "cmu440", "12x")
    assert r.returncode == 2 and r.stdout == "12x is not a number.\n"
    r = run("minehip-search", "cmu440", "18446744073709551616")  # > MaxUint64, like ParseUint
    assert r.returncode == 2


@pytest.mark.gpu
def test_search_cli_prints_client_result(gpu):
    r = run("minehip-search", "cmu440", "9999999")
    assert r.returncode == 0, r.stderr
    assert r.stdout == "Result 1228377698034 1067492\n"


@pytest.mark.gpu
def test_miner_cli_json_lines(gpu):
    lines = "\n".join([
        '{"Type":0,"Data":"","Lower":0,"Upper":0,"Hash":0,"Nonce":0}',          # Join: ignored
        '{"Type":1,"Data":"cmu440","Lower":0,"Upper":9999999,"Hash":0,"Nonce":0}',
        'garbage',                                                               # ignored
        '{"Type":1,"Data":"cmu440","Lower":9,"Upper":3}',                        # Lower > Upper: ignored
        '{"Type":1,"Data":"","Lower":0,"Upper":0}',
    ]) + "\n"
    r = run("minehip-miner", "--stdio", stdin=lines)
    assert r.returncode == 0, r.stderr
    out = r.stdout.splitlines()
    assert out[0] == '{"Type":2,"Data":"","Lower":0,"Upper":0,"Hash":1228377698034,"Nonce":1067492}'
    assert out[1] == '{"Type":2,"Data":"","Lower":0,"Upper":0,"Hash":17297653956949303043,"Nonce":0}'
    assert len(out) == 2
