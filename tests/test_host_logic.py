"""CPU tests of the host logic: the planner + the kernels' per-thread code
replayed on the host by tools/p1emu (layout coverage without a GPU), the
C-ABI library's exports, and the sharding/combine rules of the multi-GPU
path."""
import os
import random
import re
import subprocess

import pytest

from conftest import ROOT, host_bin

U64_MAX = (1 << 64) - 1
EMU = host_bin(os.path.join(ROOT, "tools", "p1emu"))


def emu(msg, lo, hi, generic=False, minthreads=None, nosplit=False, variants=None, notable=False):
    args = [EMU, msg.hex() if msg else "-", str(lo), str(hi)] + (["generic"] if generic else [])
    if minthreads is not None:
        args.append(f"minthreads={minthreads}")
    if nosplit:
        args.append("nosplit")
    if notable:
        args.append("notable")
    out = subprocess.run(args, capture_output=True, text=True, check=True).stdout.split()
    if variants is not None and out[4] != "-":
        variants.update(tuple(int(x) for x in v.split(":")) for v in out[4].split(","))
    return (int(out[0]), int(out[1])), int(out[2]), int(out[3])


def all_variants(plain_mode2):
    """(FV, MODE, TRAIL) of every P1_CASE in fast_variants.inc; the mode-2
    block is compiled only with -DP1_NV2_PLAIN (p1emu is)."""
    with open(os.path.join(ROOT, "p1_amd", "csrc", "fast_variants.inc")) as f:
        text = f.read()
    if not plain_mode2:
        text = text.split("#ifdef P1_NV2_PLAIN")[0]
    return {(int(a), int(b), 1 if c == "true" else 0)
            for a, b, c in re.findall(r"P1_CASE\((\d+), (\d+), (true|false)\)", text)}


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(EMU):
        subprocess.run(["make", "-s", "-C", ROOT, "tools/p1emu"], check=True)


def test_emu_golden_scans(golden):
    n_fast = 0
    for v in golden["scan"]:
        if v.get("large") or v["upper"] - v["lower"] > 200000:
            continue
        got, nf, _ = emu(bytes.fromhex(v["msg_hex"]), v["lower"], v["upper"])
        n_fast += nf
        assert got == (v["hash"], v["nonce"]), v
    assert n_fast > 50  # the fast (per-thread 10^k loop) path was exercised


def test_emu_generic_only_matches(golden):
    for v in golden["scan"][:40]:
        if v.get("large") or v["upper"] - v["lower"] > 20000:
            continue
        got, nf, ng = emu(bytes.fromhex(v["msg_hex"]), v["lower"], v["upper"], generic=True)
        assert nf == 0
        assert got == (v["hash"], v["nonce"]), v


def test_emu_every_layout(oracle_mod):
    """Every prefix length mod 64 x several digit counts: hits every
    (FV, NV, TRAIL) variant, PRE blocks and the k=1/2 straddle case."""
    rnd = random.Random(7)
    for L in range(0, 128):
        m = bytes(rnd.randrange(32, 127) for _ in range(L))
        for d in (5, 9, 10, 11, 20):
            b = 10 ** (d - 1)
            lo = b + rnd.randrange(0, 10**4)
            hi = min(lo + 1999, U64_MAX)
            got, nf, _ = emu(m, lo, hi)
            assert nf >= 1
            assert got == oracle_mod.scan(m, lo, hi, threads=8), (L, d, lo, hi)


@pytest.mark.parametrize("nosplit,notable", [(False, False), (True, False), (False, True)],
                         ids=["split", "plain2", "notable"])
def test_emu_every_layout_k3(oracle_mod, nosplit, notable):
    """Planner occupancy floor at 1 thread: k = 3 on small ranges, so every
    (FV, MODE, TRAIL) variant, PRE/TRAIL at k = 3 and the tens/hundreds carry
    deltas (dt/dhd) are replayed against the oracle.  The
    default pass runs the split modes 3/4 for straddling lo digits (what the
    library ships); the plain2 pass runs mode 2 (both words per nonce).  Both
    must reach every variant they can select."""
    rnd = random.Random(8)
    seen = set()
    for L in range(0, 128):
        m = bytes(rnd.randrange(32, 127) for _ in range(L))
        for d in (4, 5, 9, 10, 11, 12, 20):
            b = 10 ** (d - 1)
            # d = 4 with (L + 1) % 64 == 0 is the 1-block <0,1> layout
            lo = b + rnd.randrange(0, 3000 if d == 4 else 10**4) if d < 20 else b
            # a MODE 5 layout with 4 / 5 digits in tail block 1 covers 10^4 /
            # 10^5 nonces per hi: give it two whole blocks
            q = (L + 1) % 64 + d - 1
            hi = min(lo + {67: 24999, 68: 219999}.get(q, 4999), U64_MAX)
            got, nf, _ = emu(m, lo, hi, minthreads=1, nosplit=nosplit, variants=seen, notable=notable)
            # 6 or 7 digits in tail block 1: MODE 5 needs 10^6 / 10^7-aligned
            # blocks, too many nonces for the host replay (GPU-tested instead)
            assert nf >= 1 or (q >= 69 and not notable)
            assert got == oracle_mod.scan(m, lo, hi, threads=8), (L, d, lo, hi)
    # modes 1 and 6 run in every pass, MODEs 5 and 7 (tabulated tail block 1)
    # unless notable; modes 3/4 only with split, mode 2 only with nosplit.  Two
    # variants are out of reach at k = 3: <13,1> needs k = 2 (lo digits at
    # bytes 53, 54; at k = 3 they start at byte 52: mode 6), and <0,6> is a
    # PRE layout with lo digits at bytes 64..66, which is MODE 5 unless notable.
    def reachable(v):
        if v == (13, 1, 0) or (v == (0, 6, 0) and not notable):
            return False
        if v[1] in (1, 6):
            return True
        if v[1] in (5, 7):  # tabulated tail block 1
            return not notable
        return (v[1] == 2) == nosplit
    want = {v for v in all_variants(True) if reachable(v)}
    assert seen == want, sorted(want ^ seen)


def test_emu_every_layout_k2(oracle_mod):
    """Occupancy floor 200 on 30,000-nonce ranges: the planner lowers k to 2
    (100 nonces per thread), the only way to reach <13,1> (lo digits at bytes
    53, 54) and the k = 2 deltas of every other layout; against the oracle."""
    rnd = random.Random(9)
    seen = set()
    for L in range(0, 128):
        m = bytes(rnd.randrange(32, 127) for _ in range(L))
        for d in (9, 10, 12):
            lo = 10 ** (d - 1) + rnd.randrange(0, 10**5)
            hi = lo + 29999
            got, nf, _ = emu(m, lo, hi, minthreads=200, variants=seen)
            assert nf >= 1
            assert got == oracle_mod.scan(m, lo, hi, threads=8), (L, d, lo, hi)
    assert (13, 1, 0) in seen
    assert {v[1] for v in seen} >= {1, 4, 6}  # mode 3 (hundreds alone in word FV) needs k = 3


def _variant_cost_table():
    with open(os.path.join(ROOT, "p1_amd", "csrc", "fast_variants.inc")) as f:
        shipped = {(int(a), int(b), c == "true")
                   for a, b, c in re.findall(r"P1_CASE\((\d+), (\d+), (true|false)\)", f.read().split("#ifdef")[0])}
    with open(os.path.join(ROOT, "p1_amd", "csrc", "variant_cost.inc")) as f:
        table = {(int(a), int(b), c == "true"): (int(x), int(y))
                 for a, b, c, x, y in re.findall(r"P1_COST\((\d+), (\d+), (true|false), (\d+), (\d+)\)", f.read())}
    return shipped, table


def test_variant_cost_table_covers_shipped_variants():
    """plan_shards prices every variant the library can run."""
    shipped, table = _variant_cost_table()
    assert shipped <= set(table), sorted(shipped - set(table))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 9])
def test_plan_shards_contiguous_cover(n):
    """p1hip_plan_shards (host only): shards in order, contiguous, exactly
    [lower, upper]; empty shards only when there are fewer nonces than
    shards; lower > upper gives all-empty."""
    import p1_amd

    rnd = random.Random(n)
    cases = [(b"bradfitz", 0, 2**38 - 1), (b"cmu440-p1-" * 12, 0, 2**34 - 1), (b"", 0, U64_MAX),
             (b"msg", U64_MAX - 5, U64_MAX), (b"msg", 0, 0), (b"msg", 3, 5), (b"x" * 63, 99, 10**12 + 7)]
    cases += [(bytes(rnd.randrange(256) for _ in range(rnd.randrange(200))),) +
              tuple(sorted((rnd.randrange(2**64), rnd.randrange(2**64)))) for _ in range(20)]
    for msg, lo, hi in cases:
        shards = p1_amd.plan_shards(msg, lo, hi, n)
        assert len(shards) == n
        got = [s for s in shards if s is not None]
        assert got[0][0] == lo and got[-1][1] == hi
        for (a, b), (c, _) in zip(got, got[1:]):
            assert a <= b and c == b + 1
        if hi - lo + 1 >= n:
            assert len(got) == n
    assert p1_amd.plan_shards(b"msg", 7, 6, 3) == [None, None, None]


def test_plan_shards_cost_balance():
    """configs[3] over 8 shards: the d = 11 decade runs variant <4,1>, d = 12
    runs <4,4> (fewer loop instructions per nonce), so the planned shards
    inside d = 11 hold fewer nonces than those inside d = 12, in the ratio of
    the variants' predicted loop cycles (A 4.37 + B 2.66 per instruction)."""
    import p1_amd

    _, table = _variant_cost_table()
    cyc = {v: a * 4.37 + b * 2.66 for v, (a, b) in table.items()}
    shards = p1_amd.plan_shards(b"bradfitz", 0, 2**38 - 1, 8)
    size = [b - a + 1 for a, b in shards]
    assert sum(size) == 2**38
    assert 10**10 <= shards[1][0] and shards[1][1] < 10**11      # all d = 11
    assert 10**11 <= shards[5][0]                                 # all d = 12
    want = cyc[(4, 4, False)] / cyc[(4, 1, False)]
    assert abs(size[1] / size[5] - want) < 2e-3
    assert size[1] < 2**35 < size[5]


def test_emu_range_top(oracle_mod):
    for m in (b"msg", b"x" * 60):
        got, _, _ = emu(m, U64_MAX - 2500, U64_MAX)
        assert got == oracle_mod.scan(m, U64_MAX - 2500, U64_MAX, threads=8)


def test_emu_empty_range():
    got, nf, ng = emu(b"bradfitz", 10, 9)
    assert got == (U64_MAX, 0) and nf == 0 and ng == 0


def _header_symbols():
    with open(os.path.join(ROOT, "include", "p1hip.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(p1hip_[a-z_]+)\s*\(", text)))


def test_capi_exports_every_header_symbol():
    """libp1hip.so loads on a CPU-only host and exports every declared entry
    point (no compute call is made here)."""
    import ctypes

    import p1_amd
    from p1_amd import _lib

    lib = ctypes.CDLL(p1_amd.lib_path())
    syms = _header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == syms
    assert p1_amd.version().startswith("p1hip")


def test_capi_abi_version_and_comm_info_without_devices():
    """ADVICE r04 (struct layout): the library reports the header's
    P1HIP_ABI_VERSION and the binding refuses another one; comm_info on a
    device that is not open is an argument error, never a made-up size."""
    import p1_amd

    with open(os.path.join(ROOT, "include", "p1hip.h")) as f:
        want = int(re.search(r"#define P1HIP_ABI_VERSION (\d+)", f.read()).group(1))
    assert p1_amd.abi_version() == want == p1_amd.ABI_VERSION
    with pytest.raises(p1_amd.P1HipError) as ei:
        p1_amd.comm_info(0)
    assert ei.value.rc == -4


def test_library_registers_no_exit_time_destructor():
    """nothing of libp1hip.so runs at process exit that
    could free device memory after the ROCm runtime is gone.  The runtime
    singleton is never destroyed (p1hip.hip rt()), so the library registers
    no process-exit destructor (__cxa_atexit); the only exit-time code left
    is the thread_local error strings' (__cxa_thread_atexit, host memory)."""
    import shutil

    objdump = shutil.which("objdump")
    if not objdump:
        pytest.skip("binutils objdump not present")
    import p1_amd

    dis = subprocess.run([objdump, "-d", p1_amd.lib_path()], capture_output=True, text=True, check=True).stdout
    calls = re.findall(r"call\s+\S+\s+<(__cxa_\w*atexit)@plt>", dis)
    assert calls and set(calls) == {"__cxa_thread_atexit"}, sorted(set(calls))


def test_capi_no_device_fails_loudly():
    """Without a GPU the product path raises; it never falls back to a CPU hash."""
    import p1_amd

    try:
        import torch

        if torch.cuda.device_count() > 0:
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(p1_amd.P1HipError) as ei:
        p1_amd.scan("bradfitz", 0, 10)
    assert ei.value.rc == -1


def test_capi_bad_args():
    import ctypes

    import p1_amd

    lib = p1_amd.load()
    h, n = ctypes.c_uint64(), ctypes.c_uint64()
    assert lib.p1hip_scan(None, 5, 0, 1, ctypes.byref(h), ctypes.byref(n)) == -4
    assert lib.p1hip_scan(b"x", (1 << 28) + 1, 0, 1, ctypes.byref(h), ctypes.byref(n)) == -4


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_range_covers(world):
    from p1_amd import shard_range

    for lo, hi in [(0, 0), (0, 9), (5, 3), (0, (1 << 32) - 1), (U64_MAX - 5, U64_MAX), (0, U64_MAX)]:
        shards = [shard_range(lo, hi, r, world) for r in range(world)]
        got = [s for s in shards if s is not None]
        if lo > hi:
            assert not got
            continue
        assert got[0][0] == lo and got[-1][1] == hi
        for a, b in zip(got, got[1:]):
            assert b[0] == a[1] + 1
        sizes = [b - a + 1 for a, b in got]
        assert max(sizes) - min(sizes) <= 1


def test_combine_keys_rules():
    from p1_amd import combine_keys

    assert combine_keys([]) == (U64_MAX, 0)
    assert combine_keys([(U64_MAX, 0), (U64_MAX, 0)]) == (U64_MAX, 0)
    assert combine_keys([(5, 9), (5, 3), (7, 1)]) == (5, 3)
    assert combine_keys([(U64_MAX, 0), (U64_MAX - 1, 12)]) == (U64_MAX - 1, 12)


def test_sharded_oracle_equals_serial(oracle_mod):
    from p1_amd import combine_keys, shard_range

    for world in (2, 4, 8):
        for lo, hi in [(0, 9999), (10**9 - 3000, 10**9 + 3000)]:
            keys = []
            for r in range(world):
                s = shard_range(lo, hi, r, world)
                if s:
                    keys.append(oracle_mod.scan("bradfitz", s[0], s[1]))
            assert combine_keys(keys) == oracle_mod.scan("bradfitz", lo, hi)


def test_emu_every_tail_layout(oracle_mod):
    """Exhaustive over the tail layout: every (L + 1) % 64 = r in 0..63 x
    every digit count d in 4..20 (the layout -- which bytes hold which
    digit, B_tail, the variant and k -- depends only on r and d), with and
    without a midstate block, at k = 3 (occupancy floor 1), against the
    oracle.  MODE 5 with 6 or 7 digits in tail block 1 needs 10^6 / 10^7-
    aligned blocks, too many for the host replay: those run their ragged
    edges only (the GPU test runs the blocks)."""
    import concurrent.futures as cf

    rnd = random.Random(10)
    cases = []
    for r in range(64):
        for d in range(4, 21):
            L = (r - 1) % 64 + 64 * rnd.randrange(0, 2)
            m = bytes(rnd.randrange(32, 127) for _ in range(L))
            q = r + d - 1
            lo = 10 ** (d - 1) + rnd.randrange(0, 10**4)
            hi = min(lo + {67: 24999, 68: 219999}.get(q, 4999), U64_MAX)
            cases.append((m, lo, hi))

    def run(c):
        m, lo, hi = c
        return emu(m, lo, hi, minthreads=1)[0] == oracle_mod.scan(m, lo, hi, threads=1), c

    with cf.ThreadPoolExecutor(8) as ex:
        bad = [c for ok, c in ex.map(run, cases) if not ok]
    assert not bad, bad[:3]


@pytest.mark.parametrize("k", [1, 2])
def test_emu_every_tail_layout_small_k(oracle_mod, k):
    """The exhaustive (r, d) grid at k = 2 and 1 (occupancy floor 200 on
    ranges of 3 x 10^(k+2) nonces), replayed on the CPU against the oracle."""
    import concurrent.futures as cf

    rnd = random.Random(11 + k)
    span = 3 * 10 ** (k + 2)
    cases = []
    for r in range(64):
        for d in range(4, 21):
            L = (r - 1) % 64 + 64 * rnd.randrange(0, 2)
            m = bytes(rnd.randrange(32, 127) for _ in range(L))
            lo = 10 ** (d - 1) + rnd.randrange(0, 10**5)
            cases.append((m, lo, lo + span - 1))

    def run(c):
        m, lo, hi = c
        return emu(m, lo, hi, minthreads=200)[0] == oracle_mod.scan(m, lo, hi, threads=1), c

    with cf.ThreadPoolExecutor(8) as ex:
        bad = [c for ok, c in ex.map(run, cases) if not ok]
    assert not bad, bad[:3]
