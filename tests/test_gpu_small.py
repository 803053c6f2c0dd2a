"""GPU parity of the small-scan path: shares of at most 2^16 nonces run as one
k_scan_small launch (plan in the kernel arguments, generic kernel, partials
folded by the last workgroup through an agent-scope ticket, result written
to pinned host memory).  It is what configs[0]'s request (`bradfitz [0,
9999]`) and every p1hip_hash take in production.

Checked bit-exact against the oracle and the golden fixtures, on every
message length and digit count, across decade boundaries, at the size limit
(2^16 in, 2^16 + 1 out), at the top of the u64 range, over many consecutive
scans (the ticket must be back at 0 after each), and on two devices (host
combine and a one-device RCCL communicator).

Reference: miner.go:56-63 (scan), hash.go:13-17 (Hash)."""
import random
import statistics
import time

import pytest

pytestmark = pytest.mark.gpu
U64_MAX = (1 << 64) - 1
SMALL = 1 << 16


@pytest.fixture
def small(gpu, monkeypatch):
    monkeypatch.setenv("P1HIP_SMALL_MAX_NONCES", str(SMALL))
    gpu.reset_stats()
    yield gpu
    monkeypatch.setenv("P1HIP_SMALL_MAX_NONCES", "0")


def test_small_kats_and_config1(small):
    assert small.hash("msg", 0) == 13781283048668101583
    assert small.hash("msg", 1) == 4754799531757243342
    assert small.hash("msg", 2) == 5611725180048225792
    assert small.scan("msg", 0, 2) == (4754799531757243342, 1)
    assert small.scan("bradfitz", 0, 9999) == (1419516646206828, 9898)
    s = small.get_stats()
    assert s["small_scans"] == s["scans"] == 5 and s["fast_nonces"] == 0


def test_small_golden(small, golden):
    n = 0
    for v in golden["hash"]:
        assert small.hash(bytes.fromhex(v["msg_hex"]), v["nonce"]) == v["hash"], v
        n += 1
    for v in golden["scan"]:
        if v["lower"] <= v["upper"] and v["upper"] - v["lower"] < SMALL:
            got = small.scan(bytes.fromhex(v["msg_hex"]), v["lower"], v["upper"])
            assert got == (v["hash"], v["nonce"]), v
            n += 1
    assert small.get_stats()["small_scans"] == n


def test_small_every_length_and_decade(small, oracle_mod):
    rnd = random.Random(61)
    for L in range(0, 130):
        m = bytes(rnd.randrange(32, 127) for _ in range(L))
        for d in (1, 3, 5, 8, 10, 11, 15, 20):
            b = 10 ** (d - 1)
            lo = max(0, b - rnd.randrange(0, 300))  # mostly straddles a decade
            hi = min(lo + rnd.randrange(0, 3000), U64_MAX)
            assert small.scan(m, lo, hi) == oracle_mod.scan(m, lo, hi, threads=8), (L, d, lo, hi)


def test_small_size_limit(small, oracle_mod):
    for lo, hi, is_small in ((0, SMALL - 1, True), (0, SMALL, False), (10**9 - 40000, 10**9 + SMALL - 40001, True)):
        small.reset_stats()
        got = small.scan("bradfitz", lo, hi)
        assert got == oracle_mod.scan(b"bradfitz", lo, hi, threads=8), (lo, hi)
        assert small.get_stats()["small_scans"] == (1 if is_small else 0)


def test_small_edges(small, oracle_mod):
    for m in (b"", b"msg", b"x" * 55, b"y" * 119):
        for lo, hi in ((U64_MAX - 5000, U64_MAX), (U64_MAX, U64_MAX), (0, 0), (9, 10), (99, 100)):
            assert small.scan(m, lo, hi) == oracle_mod.scan(m, lo, hi, threads=8), (m, lo, hi)
    assert small.scan("msg", 5, 4) == (U64_MAX, 0)


def test_small_many_consecutive(small, oracle_mod):
    """The last-workgroup ticket is reset by the kernel itself: 300 scans in
    a row of random sizes (1 to 2^16 nonces, 1 to 256 workgroups)."""
    rnd = random.Random(62)
    for i in range(300):
        lo = rnd.choice([0, rnd.randrange(10**6), rnd.randrange(10**12), rnd.randrange(U64_MAX - SMALL)])
        hi = lo + rnd.choice([0, 1, 255, 256, 257, rnd.randrange(SMALL)])
        m = b"bradfitz" if i % 2 else b"cmu440-p1-" * 12
        assert small.scan(m, lo, hi) == oracle_mod.scan(m, lo, hi, threads=8), (i, lo, hi)
    assert small.get_stats()["small_scans"] == 300


def test_small_latency_recorded(small, capsys):
    for _ in range(5):
        small.scan("bradfitz", 0, 9999)
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        assert small.scan("bradfitz", 0, 9999) == (1419516646206828, 9898)
        ts.append((time.perf_counter() - t0) * 1e6)
    with capsys.disabled():
        print(f"\nconfigs[0] request via the small path: median {statistics.median(ts):.1f} us, "
              f"min {min(ts):.1f} us over 50 calls")


@pytest.mark.parametrize("knob", ["P1HIP_NO_RCCL", "P1HIP_FORCE_RCCL"])
def test_small_multi_device(small, oracle_mod, monkeypatch, knob):
    """Two shards on GPU 0 listed twice with a host combine, and one device
    with an RCCL communicator: the small path leaves each device's key in
    device memory for the combine."""
    monkeypatch.setenv(knob, "1")
    ords = [0, 0] if knob == "P1HIP_NO_RCCL" else [0]
    small.shutdown()
    small.init_devices(ords)
    try:
        rnd = random.Random(63)
        for _ in range(30):
            lo = rnd.randrange(10**10)
            hi = lo + rnd.randrange(2 * SMALL)
            assert small.scan("bradfitz", lo, hi) == oracle_mod.scan(b"bradfitz", lo, hi, threads=8)
        assert small.scan("bradfitz", 0, 9999) == (1419516646206828, 9898)
    finally:
        monkeypatch.delenv(knob)
        small.shutdown()
        small.init_devices([0])
