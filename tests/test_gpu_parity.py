"""GPU parity: libp1hip.so (through its C ABI) against the oracle and the
golden fixtures.  Integer work -> bit-exact equality everywhere.

Reference: miner.go:56-63 (scan), hash.go:13-17 (Hash)."""
import random

import pytest

pytestmark = pytest.mark.gpu
U64_MAX = (1 << 64) - 1
M120 = b"cmu440-p1-" * 12


def test_handout_kats(gpu):
    assert gpu.hash("msg", 0) == 13781283048668101583
    assert gpu.hash("msg", 1) == 4754799531757243342
    assert gpu.hash("msg", 2) == 5611725180048225792
    assert gpu.scan("msg", 0, 2) == (4754799531757243342, 1)


def test_config1_client_answer(gpu):
    # configs[0]: client 'bradfitz' maxNonce 9999 prints "Result 1419516646206828 9898"
    assert gpu.scan("bradfitz", 0, 9999) == (1419516646206828, 9898)


def test_golden_hashes(gpu, golden):
    for v in golden["hash"]:
        assert gpu.hash(bytes.fromhex(v["msg_hex"]), v["nonce"]) == v["hash"], v


def test_golden_scans(gpu, golden):
    for v in golden["scan"]:
        got = gpu.scan(bytes.fromhex(v["msg_hex"]), v["lower"], v["upper"])
        assert got == (v["hash"], v["nonce"]), v


def test_config2_full_range(gpu):
    # configs[1]: 'bradfitz', [0, 2^32) -- answer from SURVEY.md 8(c) (hashlib, 8 processes)
    assert gpu.scan("bradfitz", 0, (1 << 32) - 1) == (5256245051, 1626825724)


def test_every_layout_vs_oracle(gpu, oracle_mod):
    rnd = random.Random(11)
    for L in range(0, 130):
        m = bytes(rnd.randrange(32, 127) for _ in range(L))
        for d in (4, 7, 10, 11, 15, 20):
            b = 10 ** (d - 1)
            lo = b + rnd.randrange(0, 10**4) if d < 20 else b
            hi = min(lo + rnd.randrange(1500, 4000), U64_MAX)
            assert gpu.scan(m, lo, hi) == oracle_mod.scan(m, lo, hi, threads=8), (L, d, lo, hi)


def test_decade_straddles_vs_oracle(gpu, oracle_mod):
    rnd = random.Random(12)
    for L in (0, 8, 45, 54, 55, 62, 63, 64, 119, 120, 1000):
        m = bytes(rnd.randrange(32, 127) for _ in range(L))
        for d in range(2, 20):
            b = 10 ** (d - 1)
            lo, hi = max(0, b - 1234), b + 2345
            assert gpu.scan(m, lo, hi) == oracle_mod.scan(m, lo, hi, threads=8), (L, d)


def test_larger_ranges_vs_oracle(gpu, oracle_mod):
    for m, lo, hi in [(b"bradfitz", 0, 999_999), (M120, 10**9 - 500_000, 10**9 + 500_000),
                      (b"x" * 55, 12_345_678, 13_045_678), (b"", 0, 1_000_000)]:
        assert gpu.scan(m, lo, hi) == oracle_mod.scan(m, lo, hi, threads=8), (m[:8], lo, hi)


def test_edges(gpu, oracle_mod):
    assert gpu.scan("bradfitz", 5, 3) == (U64_MAX, 0)            # Lower > Upper
    assert gpu.scan("bradfitz", 0, 0) == (oracle_mod.hash("bradfitz", 0), 0)
    assert gpu.scan(b"", 7, 7) == (oracle_mod.hash(b"", 7), 7)
    for lo in (U64_MAX - 3000, U64_MAX):                           # no wrap at 2^64-1
        assert gpu.scan("msg", lo, U64_MAX) == oracle_mod.scan("msg", lo, U64_MAX, threads=8)
    big = bytes(range(256)) * 6                                     # 1536 B, > LSP frame
    assert gpu.scan(big, 10**12, 10**12 + 3000) == oracle_mod.scan(big, 10**12, 10**12 + 3000, threads=8)
    utf8 = "héllo wörld ✓".encode()
    assert gpu.scan(utf8, 0, 5000) == oracle_mod.scan(utf8, 0, 5000, threads=8)


def test_tie_breaking_reduction(gpu):
    rnd = random.Random(5)
    # equal minimum hashes: lowest nonce wins (strict '<' at miner.go:59)
    n = 100_000
    hs = [rnd.randrange(1 << 40, U64_MAX) for _ in range(n)]
    ns = list(range(10**6, 10**6 + n))
    rnd.shuffle(ns)
    pos = rnd.sample(range(n), 7)
    for p in pos:
        hs[p] = 12345
    want = (12345, min(ns[p] for p in pos))
    assert gpu.reduce_pairs(hs, ns) == want
    # ties inside one wave and across waves / workgroups
    for size in (1, 2, 63, 64, 65, 255, 256, 257, 4097):
        hs = [7] * size
        ns = list(range(size, 0, -1))
        assert gpu.reduce_pairs(hs, ns) == (7, 1)
    # identity rules
    assert gpu.reduce_pairs([], []) == (U64_MAX, 0)
    assert gpu.reduce_pairs([U64_MAX] * 300, list(range(5, 305))) == (U64_MAX, 0)
    assert gpu.reduce_pairs([U64_MAX, U64_MAX - 1], [1, 99]) == (U64_MAX - 1, 99)


def test_full_size_config3_exact(gpu, oracle_mod, large):
    """configs[2] (120-byte msg, [0, 2^34)): equal to the exact answer pinned
    by tools/pin_large.c (independent CPU restatement, tests/golden), plus the
    size-independent properties: the reported nonce re-hashes to the reported
    hash, and the scan is the min of its two halves (split at an arbitrary
    point), each of which also re-hashes."""
    hi = (1 << 34) - 1
    h, n = gpu.scan(M120, 0, hi)
    assert (h, n) == large[(M120, 0, hi)]
    assert 0 <= n <= hi and oracle_mod.hash(M120, n) == h
    cut = 9_876_543_210
    a = gpu.scan(M120, 0, cut)
    b = gpu.scan(M120, cut + 1, hi)
    assert min(a, b) == (h, n)
    for hh, nn in (a, b):
        assert oracle_mod.hash(M120, nn) == hh


def test_stats_and_profiling(gpu):
    gpu.reset_stats()
    gpu.set_profiling(True)
    gpu.scan("bradfitz", 0, 10**8)
    s = gpu.get_stats()
    gpu.set_profiling(False)
    assert s["scans"] == 1 and s["fast_launches"] >= 1 and s["scan_launches"] == 1
    assert s["fast_nonces"] + s["generic_nonces"] == 10**8 + 1 == s["scan_nonces"]
    assert s["scan_kernel_ms"] > 0
    assert s["fast_alg_ops"] == 1384 * s["fast_nonces"]  # 'bradfitz' is 1 block per nonce
    assert s["scan_alg_ops"] == 1384 * s["scan_nonces"]


def test_init_variants(gpu):
    got = gpu.init(1)
    assert got == 1 and gpu.device_count() == 1
    gpu.init_devices([0])
    assert gpu.scan("msg", 0, 2) == (4754799531757243342, 1)


def test_multi_device_path_on_one_gpu(gpu, oracle_mod, monkeypatch):
    """p1hip_scan's multi-device code path (one host thread per device,
    contiguous shards, combine) with GPU 0 listed three times; RCCL cannot
    pair a GPU with itself, so the test combines through the host
    (P1HIP_NO_RCCL=1, read at init)."""
    monkeypatch.setenv("P1HIP_NO_RCCL", "1")
    try:
        gpu.init_devices([0, 0, 0])
        assert gpu.device_count() == 3
        for m, lo, hi in [(b"bradfitz", 0, 9999), (b"x" * 57, 10**9 - 4000, 10**9 + 4000),
                          (b"msg", 0, 1), (b"msg", 5, 5), (b"msg", 9, 3)]:
            assert gpu.scan(m, lo, hi) == oracle_mod.scan(m, lo, hi, threads=8), (m, lo, hi)
        assert gpu.scan("bradfitz", 0, (1 << 32) - 1) == (5256245051, 1626825724)
        # MODE 5 on every "device" (each builds and caches its own K+W table),
        # shards cut by p1hip_plan_shards
        c3 = (b"cmu440-p1-" * 12, 10**10 - 2 * 10**9, 10**10 + 4 * 10**9)
        got3 = gpu.scan(*c3)
    finally:
        monkeypatch.delenv("P1HIP_NO_RCCL")
        gpu.init_devices([0])
    assert got3 == gpu.scan(*c3)
    assert oracle_mod.hash(c3[0], got3[1]) == got3[0]


def test_long_messages_and_limits(gpu, oracle_mod):
    import ctypes

    m = bytes((i * 131 + 7) % 251 for i in range(1 << 20))  # 1 MiB: 16384 midstate blocks on the host
    for lo, hi in [(0, 3000), (10**11 - 1500, 10**11 + 1500)]:
        assert gpu.scan(m, lo, hi) == oracle_mod.scan(m, lo, hi, threads=8)
    lib = gpu.load()
    h, n = ctypes.c_uint64(), ctypes.c_uint64()
    assert lib.p1hip_scan(b"x", (1 << 28) + 1, 0, 1, ctypes.byref(h), ctypes.byref(n)) == -4


def test_random_requests_vs_oracle(gpu, oracle_mod):
    """Many small random requests (random bytes incl. non-UTF-8, random
    lengths and ranges anywhere in u64), the way a server would send them."""
    rnd = random.Random(2026)
    for _ in range(300):
        L = rnd.choice([rnd.randrange(0, 140), rnd.randrange(0, 2000)])
        m = bytes(rnd.randrange(0, 256) for _ in range(L))
        lo = max(0, rnd.choice([rnd.randrange(0, 10**6), rnd.randrange(0, U64_MAX),
                                10 ** rnd.randrange(1, 20) - rnd.randrange(0, 500)]))
        hi = min(lo + rnd.randrange(0, 3000), U64_MAX)
        assert gpu.scan(m, lo, hi) == oracle_mod.scan(m, lo, hi, threads=8), (L, lo, hi)


def test_reduce_pairs_large(gpu):
    rnd = random.Random(9)
    n = 1_000_003
    hs = [rnd.randrange(0, U64_MAX) for _ in range(n)]
    ns = [rnd.randrange(0, U64_MAX) for _ in range(n)]
    want = min(zip(hs, ns))
    assert gpu.reduce_pairs(hs, ns) == want


def test_config4_range_on_one_gpu_multi_batch(gpu, oracle_mod, monkeypatch, large):
    """configs[3]'s whole [0, 2^38) on one GPU (~1.07M workgroups): one
    launch by default, and several launches (batches) under a 2^19-workgroup
    cap (test knob P1HIP_MAX_LAUNCH_BLOCKS, read per scan).  Both equal the
    exact answer pinned by tools/pin_large.c; also the size-independent
    properties: the result re-hashes on the oracle and equals the min of two
    independently scanned halves."""
    hi = (1 << 38) - 1
    gpu.reset_stats()
    h, n = gpu.scan("bradfitz", 0, hi)
    assert (h, n) == large[(b"bradfitz", 0, hi)]
    assert gpu.get_stats()["scan_launches"] == 1
    assert oracle_mod.hash("bradfitz", n) == h
    monkeypatch.setenv("P1HIP_MAX_LAUNCH_BLOCKS", str(1 << 19))
    gpu.reset_stats()
    assert gpu.scan("bradfitz", 0, hi) == (h, n)
    assert gpu.get_stats()["scan_launches"] >= 2
    monkeypatch.delenv("P1HIP_MAX_LAUNCH_BLOCKS")
    a = gpu.scan("bradfitz", 0, (1 << 37) - 1)
    b = gpu.scan("bradfitz", 1 << 37, hi)
    assert min(a, b) == (h, n)


def test_share_in_pieces(gpu, oracle_mod, monkeypatch):
    """A device's share is scanned in pieces of at most 2^40 nonces (the plan
    of one piece stays small however large the request); forced here to
    pieces of 10^6 + 7 nonces, the answer and the nonce count are those of
    the one-piece scan."""
    cases = [("bradfitz", 10**9 - 3 * 10**6, 10**9 + 5 * 10**6), (b"cmu440-p1-" * 12, 10**10, 10**10 + 9 * 10**6)]
    want = [gpu.scan(m, lo, hi) for m, lo, hi in cases]
    monkeypatch.setenv("P1HIP_MAX_SCAN_SPAN", str(10**6 + 7))
    for (m, lo, hi), w in zip(cases, want):
        gpu.reset_stats()
        assert gpu.scan(m, lo, hi) == w
        assert gpu.get_stats()["scan_nonces"] == hi - lo + 1
    monkeypatch.delenv("P1HIP_MAX_SCAN_SPAN")
    for (m, lo, hi), (h, n) in zip(cases, want):
        assert oracle_mod.hash(m, n) == h
