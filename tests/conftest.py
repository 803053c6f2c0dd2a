import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def host_bin(path):
    """A host program's path, or its sanitizer build when P1_SAN_DIR names
    one (`make sanitize`: build/san/asan, build/san/tsan; tools/sanitize.sh
    re-runs the host-program tests against those)."""
    san = os.environ.get("P1_SAN_DIR")
    if san:
        alt = os.path.join(san, os.path.basename(path))
        if os.path.exists(alt):
            return alt
    return path


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    # a fresh checkout builds once (normally everything is prebuilt by `make`)
    from p1_amd.build import ensure_built

    ensure_built()


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def large(golden):
    """Exact full-range answers of the BASELINE configs, (msg bytes, lower,
    upper) -> (hash, nonce): configs[1] from the survey's hashlib run,
    configs[2]/[3]/[4] from tools/pin_large.c (a container-only SHA-NI /
    AVX-512 restatement validated against the oracle and hashlib,
    tests/golden/pin_large_validation.json)."""
    return {(bytes.fromhex(v["msg_hex"]), v["lower"], v["upper"]): (v["hash"], v["nonce"])
            for v in golden["scan"] if v.get("large")}


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.load()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    """The HIP library, initialised on device 0.  Fails (not skips) when the
    library or the device is missing: on the GPU box that is a real failure."""
    import p1_amd

    # Shares of <= 2^16 nonces take the one-launch small path (k_scan_small,
    # generic kernel) in production.  The parity suite's small ranges are
    # there to exercise the fast kernel variants, so the session turns the
    # small path off (read per scan); tests/test_gpu_small.py turns it back on.
    os.environ["P1HIP_SMALL_MAX_NONCES"] = "0"
    # the library honours its test knobs only under this master switch
    # (production ignores them; bench.py refuses to time with it set)
    os.environ["P1HIP_TEST_KNOBS"] = "1"
    p1_amd.load()
    p1_amd.init_devices([0])
    return p1_amd
