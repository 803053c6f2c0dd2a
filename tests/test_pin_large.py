"""tools/pin_large.c -- the container-only checker that pins the exact
full-range answers of configs[2], [3] and [4] (tests/golden/golden.json
`large` vectors) -- against the oracle and hashlib, on CPU.

The full validation (10^8-nonce sub-ranges of both messages, configs[1]'s
hashlib answer over [0, 2^32)) runs in `python tools/pin_large.py validate`
and is recorded in tests/golden/pin_large_validation.json; here a shorter
version runs on every CPU suite, and the record is checked against the
tool's current source."""
import hashlib
import json
import os
import random

import pytest

from conftest import ROOT

import tools.pin_large as pin  # noqa: E402

M120 = b"cmu440-p1-" * 12


def _cpu_flags():
    try:
        return open("/proc/cpuinfo").read()
    except OSError:
        return ""


needs_sha = pytest.mark.skipif(not (" sha_ni" in _cpu_flags() and " avx512f" in _cpu_flags()),
                               reason="pin_large needs the x86 SHA extensions and AVX-512 (container CPU)")


def go_hash(m, n):
    return int.from_bytes(hashlib.sha256(m + b" " + str(n).encode()).digest()[:8], "big")


def test_validation_record_matches_tool_source(golden):
    """Runs on every CPU (no SHA extensions needed): an edited pin_large.c
    cannot leave stale pins behind, and every pin is labelled as not covered
    by a reference-held fixture."""
    rec = json.load(open(pin.VALID))
    assert rec["tool_sha16"] == pin.src_sha(), "pin_large.c changed since it was validated: re-run validate"
    assert all(c["ok"] for c in rec["checks"])
    big = [c for c in rec["checks"] if c.get("nonces", 0) >= 10**8]
    assert {c["msg_hex"] for c in big} == {b"bradfitz".hex(), M120.hex()}
    # every large golden answer came from this validated tool (or the survey's hashlib run)
    for v in golden["scan"]:
        if v.get("large") and "pin_large" in v["source"]:
            assert v["tool_sha16"] == rec["tool_sha16"] == pin.src_sha()
        if v.get("large"):
            assert v["reference_pinned"] is False and v["parity"].startswith("parity-unpinned")


@needs_sha
@pytest.mark.parametrize("sha_only", [False, True], ids=["avx512+sha", "sha-ni"])
def test_golden_scans(golden, sha_only):
    for v in golden["scan"]:
        if v.get("large") or v["upper"] - v["lower"] > 10**6:
            continue
        r, _ = pin.run(bytes.fromhex(v["msg_hex"]), v["lower"], v["upper"], threads=2, chunk_log2=16,
                       sha_only=sha_only)
        assert (r["hash"], r["nonce"]) == (v["hash"], v["nonce"]), v


@needs_sha
def test_random_hashes_vs_hashlib():
    rnd = random.Random(7)
    for _ in range(200):
        m = bytes(rnd.randrange(32, 127) for _ in range(rnd.randrange(0, 140)))
        n = rnd.randrange(0, 1 << 64)
        r, _ = pin.run(m, n, n, threads=1, chunk_log2=4)
        assert r["hash"] == go_hash(m, n), (m, n)


@pytest.mark.parametrize("m,lo,hi", [
    (b"bradfitz", (1 << 38) - 2 * 10**7, (1 << 38) - 1),        # AVX-512 blocks + SHA-NI edges, d = 12
    (b"bradfitz", 10**10 - 10**7, 10**10 + 10**7 - 1),          # decade straddle on both paths
    (M120, (1 << 34) - 5 * 10**6, (1 << 34) - 1),              # two tail blocks, cached first block
], ids=["c4-top", "bradfitz-straddle", "c3-top"])
@needs_sha
def test_subranges_vs_oracle(oracle_mod, m, lo, hi):
    want = oracle_mod.scan(m, lo, hi, threads=8)
    for sha_only in (False, True):
        r, _ = pin.run(m, lo, hi, threads=8, chunk_log2=22, sha_only=sha_only)
        assert (r["hash"], r["nonce"]) == want, sha_only


@needs_sha
def test_chunk_results_resume_from_checkpoint(tmp_path, oracle_mod):
    ck = str(tmp_path / "ck")
    lo, hi = 10**9, 10**9 + 3 * 10**6
    a, _ = pin.run(b"bradfitz", lo, hi, threads=2, chunk_log2=20, ckpt=ck)
    n_lines = len(open(ck).read().split("\n"))
    b, _ = pin.run(b"bradfitz", lo, hi, threads=2, chunk_log2=20, ckpt=ck)  # everything reused
    assert len(open(ck).read().split("\n")) == n_lines
    assert (a["hash"], a["nonce"]) == (b["hash"], b["nonce"]) == oracle_mod.scan(b"bradfitz", lo, hi, threads=8)
