import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bitcoin-miner_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")
    # build in-tree artefacts if a fresh checkout lacks them
    if not os.path.exists(os.path.join(PKG, "minehip", "libminehip.so")) or \
            not os.path.exists(os.path.join(ROOT, "oracle", "liboracle_sha256.so")):
        subprocess.run(["make", "-s", "-C", ROOT], check=True)


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_hash():
    d = load_golden("hash_vectors.json")
    return [(bytes.fromhex(m), int(n), int(h)) for m, n, h in d["vectors"]]


@pytest.fixture(scope="session")
def golden_scan():
    d = load_golden("scan_vectors.json")
    conv = lambda v: (bytes.fromhex(v["msg_hex"]), int(v["lower"]), int(v["upper"]), int(v["hash"]), int(v["nonce"]))  # noqa: E731
    return [conv(v) for v in d["small"]], [conv(v) for v in d["config1"]]


DEV_LIB = os.path.join(ROOT, "build", "dev", "libminehip.so")


def run_dev(code, timeout=120, **env):
    """Run `code` in a child Python process whose minehip package loads the dev
    build (build/dev/libminehip.so: the product sources plus the experiment and
    test hooks, `make dev`), with extra environment `env`.  The product library
    has no hooks (tests/test_abi.py::test_product_library_has_no_dev_hooks), so
    a test that injects a failure runs here.  Returns the CompletedProcess."""
    if not os.path.exists(DEV_LIB):
        pytest.fail(f"{DEV_LIB} missing: build it with `make all` (or `make dev`)")
    e = dict(os.environ, MINEHIP_LIB=DEV_LIB, **{k: str(v) for k, v in env.items()})
    pre = f"import sys; sys.path[:0] = [{ROOT!r}, {PKG!r}]\n"
    return subprocess.run([sys.executable, "-c", pre + code], env=e, capture_output=True, text=True,
                          timeout=timeout)


@pytest.fixture(scope="session")
def gpu():
    import minehip
    if minehip.device_count() < 1:
        pytest.skip("no GPU visible")
    return minehip
