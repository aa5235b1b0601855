"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

The planner, scheduler, server loop and Go-JSON codec of libminehip are
compiled with g++ -fsanitize=address,undefined together with
tests/host/fuzz_host.cpp, which drives them with randomized inputs (ranges up
to 2^64-1, arbitrary bytes, random event orders) and checks their invariants.
GPU sanitizers are not available on the MI355X pool; this covers the host side.

liblsp440 (bitcoin-miner_amd/csrc/lsp/lsp.cpp) is built with
tests/host/fuzz_lsp.cpp twice: under address,undefined and under
ThreadSanitizer (the reference's LSP tests are meant for `go test -race`).
"""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "bitcoin-miner_amd", "csrc")
SRCS = [os.path.join(CSRC, f) for f in ("plan.cpp", "sched.cpp", "server.cpp", "message.cpp")]
DRIVER = os.path.join(ROOT, "tests", "host", "fuzz_host.cpp")
LSP_SRC = os.path.join(CSRC, "lsp", "lsp.cpp")
LSP_DRIVER = os.path.join(ROOT, "tests", "host", "fuzz_lsp.cpp")


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = str(tmp_path_factory.mktemp("asan") / "fuzz_host")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-Wall", "-o", out, DRIVER] + SRCS
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return out


@pytest.mark.parametrize("seed", [440, 1, 2])
def test_host_fuzz_under_sanitizers(fuzz_bin, seed):
    # verify_asan_link_order=0: the ASan runtime need not be the first DSO loaded
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzz_bin, str(seed), "150"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "failures=0" in r.stdout
    # fast pieces whose lanes' formatted digits were checked against the kernel's nonce formula,
    # Early layouts (interleaved lanes) among them
    import re
    m = re.search(r"fast_pieces=(\d+) early_pieces=(\d+)", r.stdout)
    assert m and int(m.group(1)) > 10000 and int(m.group(2)) > 1000, r.stdout


@pytest.fixture(scope="module", params=["address,undefined", "thread"])
def lsp_fuzz_bin(request, tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    san = request.param
    out = str(tmp_path_factory.mktemp("lsp_" + san.split(",")[0]) / "fuzz_lsp")
    extra = ["-fno-sanitize-recover=undefined"] if "undefined" in san else []
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}", *extra, "-Wall",
           "-o", out, LSP_DRIVER, LSP_SRC, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return out


@pytest.mark.parametrize("seed", [440, 7])
def test_lsp_under_sanitizers(lsp_fuzz_bin, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([lsp_fuzz_bin, str(seed), "100"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "failures=0" in r.stdout and "WARNING: ThreadSanitizer" not in r.stderr


def test_scheduler_under_thread_sanitizer(tmp_path):
    """mh_sched_* from 6 miner threads + a submitter + churn (tests/host/tsan_sched.cpp)."""
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = str(tmp_path / "tsan_sched")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-Wall", "-o", out,
           os.path.join(ROOT, "tests", "host", "tsan_sched.cpp"), os.path.join(CSRC, "sched.cpp"), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    for seed in (440, 7):
        r = subprocess.run([out, str(seed)], capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
        assert "failures=0" in r.stdout and "WARNING: ThreadSanitizer" not in r.stderr


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_multi_coordinator_under_sanitizers(tmp_path, san):
    """mh_search_multi's shard coordinator (csrc/multi.cpp: rate-weighted head shards, dynamic tail,
    hand-back of a failed worker's span) and the fixed-chunk scheduler path (search_chunks) from up
    to 8 worker threads with a stand-in search that fails for random workers, and with only k of
    the workers' host threads started (tests/host/tsan_multi.cpp): the successful spans tile the
    range once, the merge is the minimum over them, and the call fails exactly when every worker
    failed or none started (MH_EINTERNAL)."""
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    out = str(tmp_path / "tsan_multi")
    extra = ["-fno-sanitize-recover=undefined"] if "undefined" in san else []
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}", *extra, "-Wall",
           "-o", out, os.path.join(ROOT, "tests", "host", "tsan_multi.cpp"), os.path.join(CSRC, "multi.cpp"),
           os.path.join(CSRC, "plan.cpp"), os.path.join(CSRC, "sched.cpp"), "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    for seed in (440, 7):
        p = subprocess.run([out, str(seed), "60"], capture_output=True, text=True, timeout=600, env=env)
        assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-6000:])
        assert "failures=0" in p.stdout and "WARNING: ThreadSanitizer" not in p.stderr
