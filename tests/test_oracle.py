"""The oracle (CPU restatement) pinned against every known answer we hold:
the handout KATs (p1.pdf 4.1), the compiled reference's mtest vectors
 and independent hashlib fixtures (tests/golden)."""
import hashlib

import pytest

U64_MAX = (1 << 64) - 1


def test_handout_kats(oracle_mod):
    # p1.pdf section 4.1: bitcoin.Hash("msg", 0/1/2)
    assert oracle_mod.hash("msg", 0) == 13781283048668101583
    assert oracle_mod.hash("msg", 1) == 4754799531757243342
    assert oracle_mod.hash("msg", 2) == 5611725180048225792
    # ... and the scan over [0, 2] picks nonce 1
    assert oracle_mod.scan("msg", 0, 2) == (4754799531757243342, 1)


def test_sha256_fips_vectors(oracle_mod):
    for data in [b"", b"abc", b"a" * 55, b"a" * 56, b"a" * 63, b"a" * 64, b"a" * 119, b"a" * 1000]:
        assert oracle_mod.sha256(data) == hashlib.sha256(data).digest()


def test_golden_hashes(oracle_mod, golden):
    for v in golden["hash"]:
        assert oracle_mod.hash(bytes.fromhex(v["msg_hex"]), v["nonce"]) == v["hash"], v


def test_golden_scans(oracle_mod, golden):
    for v in golden["scan"]:
        if v.get("large"):
            continue
        got = oracle_mod.scan(bytes.fromhex(v["msg_hex"]), v["lower"], v["upper"], threads=4)
        assert got == (v["hash"], v["nonce"]), v


def test_mtest_vectors_present(golden):
    srcs = [v for v in golden["scan"] if v["source"].startswith("mtest")]
    assert len(srcs) == 4


def test_scan_semantics(oracle_mod):
    assert oracle_mod.scan("bradfitz", 5, 3) == (U64_MAX, 0)  # Lower > Upper
    # single nonce == Hash
    assert oracle_mod.scan("bradfitz", 77, 77) == (oracle_mod.hash("bradfitz", 77), 77)
    # Upper == 2^64-1 terminates (documented divergence from the wrapping Go loop)
    h, n = oracle_mod.scan("msg", U64_MAX - 10, U64_MAX)
    assert U64_MAX - 10 <= n <= U64_MAX


@pytest.mark.parametrize("threads", [2, 3, 8])
def test_mt_equals_serial(oracle_mod, threads):
    for lo, hi in [(0, 5000), (999, 1001), (10**9 - 300, 10**9 + 300)]:
        assert oracle_mod.scan("bradfitz", lo, hi, threads) == oracle_mod.scan("bradfitz", lo, hi)
