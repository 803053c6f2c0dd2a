"""p1server: job splitting, round-robin scheduling across miner processes,
reassignment of a lost miner's chunk, lexicographic min over chunks
(server.go:83-168 + handout 4.2).  CPU tests drive it
with tests/fake_miner.py (oracle-backed test double); the GPU test with real
`p1miner serve` processes."""
import json
import os
import subprocess

import pytest

from conftest import ROOT, host_bin

SERVER = host_bin(os.path.join(ROOT, "p1_amd", "p1server"))
FAKE = f"python3 {os.path.join(ROOT, 'tests', 'fake_miner.py')}"
U64_MAX = (1 << 64) - 1


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(SERVER):
        subprocess.run(["make", "-s", "-C", ROOT, "p1_amd/p1server"], check=True)


def server(args, stdin=None, timeout=600):
    return subprocess.run([SERVER] + args, input=stdin, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("miners,chunk", [(1, 10**6), (3, 1000), (4, 333), (8, 1)])
def test_split_scan_matches_oracle(oracle_mod, miners, chunk):
    hi = 9999 if chunk > 1 else 300
    r = server(["--miners", str(miners), "--chunk", str(chunk), "--miner-cmd", FAKE, "scan", "bradfitz", "0", str(hi)])
    assert r.returncode == 0, r.stderr
    h, n = oracle_mod.scan("bradfitz", 0, hi)
    assert r.stdout.strip() == f"Result {h} {n}"


def test_lost_miner_chunk_is_reassigned(oracle_mod):
    # miner on "device" 0 dies at its 3rd request, miner 2 at its 5th; miner 1 survives
    cmd = f"FAKE_DIE_AFTER=$((2+{{dev}})) {FAKE}"
    r = server(["--miners", "3", "--devices", "0,100,3", "--chunk", "500", "--miner-cmd", cmd,
                "scan", "bradfitz", "0", "19999"])
    assert r.returncode == 0, r.stderr
    h, n = oracle_mod.scan("bradfitz", 0, 19999, threads=4)
    assert r.stdout.strip() == f"Result {h} {n}"


def test_all_miners_lost_reports_disconnected():
    cmd = f"FAKE_DIE_AFTER=1 {FAKE}"
    r = server(["--miners", "2", "--chunk", "100", "--miner-cmd", cmd, "scan", "bradfitz", "0", "9999"])
    assert r.returncode == 1 and r.stdout.strip() == "Disconnected"  # client.go:64-66


def test_serve_many_requests_in_order(oracle_mod):
    reqs = [("bradfitz", 0, 9999), ("msg", 0, 2), ("x", 9, 3), ("héllo", 10**9 - 1500, 10**9 + 1500),
            ("", 0, 0)]
    stdin = "".join(json.dumps({"Type": 1, "Data": d, "Lower": lo, "Upper": hi, "Hash": 0, "Nonce": 0},
                               ensure_ascii=False) + "\n" for d, lo, hi in reqs)
    stdin = '{"Type":0}\n' + stdin  # a Join line is ignored
    r = server(["--miners", "3", "--chunk", "700", "--miner-cmd", FAKE, "serve"], stdin)
    assert r.returncode == 0, r.stderr
    got = [json.loads(x) for x in r.stdout.strip().split("\n")]
    want = [oracle_mod.scan(d, lo, hi) for d, lo, hi in reqs]
    assert [(g["Hash"], g["Nonce"]) for g in got] == want
    assert all(g["Type"] == 2 for g in got)


def test_scheduler_unit(tmp_path):
    """scheduler.hpp on its own: the full u64 range as one cursor, lost-miner
    chunks first, identity and tie-breaking, completion order, cancelled
    clients (tests/sched_test.cpp)."""
    exe = str(tmp_path / "sched_test")
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-o", exe,
                    os.path.join(ROOT, "tests", "sched_test.cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "sched_test: ok"


def test_scheduler_randomized_simulation(tmp_path):
    """scheduler.hpp against a brute-force model under random joins, losses
    (holding a chunk, or after computing it), departed clients, stray
    Results, results out of order, empty ranges and ranges at the u64 top
    (tests/sched_sim.cpp), built with ASan + UBSan.  A stand-in hash with a
    message-dependent range makes equal minima common, so the lowest-nonce
    rule is exercised within and across chunks (dropping the requeue of a
    lost chunk, reversing the tie rule or widening a chunk by one nonce each
    fail it)."""
    exe = str(tmp_path / "sched_sim")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=undefined", "-o", exe, os.path.join(ROOT, "tests", "sched_sim.cpp")],
                   check=True)
    total = 0
    for seed in range(1, 25):
        r = subprocess.run([exe, str(seed), "3000"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and r.stdout.startswith("sched_sim: ok"), (seed, r.stdout, r.stderr[-2000:])
        total += int(r.stdout.split()[2])
    assert total > 24 * 200  # requests completed and checked


def test_usage():
    assert server([]).returncode == 2
    assert server(["--chunk", "0", "scan", "a", "0", "1"]).returncode == 2


@pytest.mark.gpu
def test_gpu_miners_split_job(oracle_mod):
    """Three real GPU miner processes (`p1miner serve`) sharing device 0."""
    r = server(["--miners", "3", "--devices", "0", "--chunk", str(10**8), "scan", "bradfitz", "0",
                str((1 << 32) - 1)])
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "Result 5256245051 1626825724"
    r = server(["--miners", "2", "--chunk", "4096", "scan", "cmu440-p1-" * 12, "0", "99999"])
    assert r.returncode == 0, r.stderr
    h, n = oracle_mod.scan("cmu440-p1-" * 12, 0, 99999, threads=8)
    assert r.stdout.strip() == f"Result {h} {n}"
