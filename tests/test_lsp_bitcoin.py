"""The bitcoin system over LSP/UDP (configs[0] and
configs[4]): `p1server lsp` splits client requests over miners that joined
with a Join message (server.go:83-168 + scheduler.hpp), miners answer over
their LSP connection (miner.go:13-73), the client prints the result
(client.go:13-66).

CPU tests use tools/lsp_fake_miner (the miner loop with the oracle instead
of the GPU; a test double); the GPU test runs configs[4] with real
`p1miner lsp` processes on GPU 0, window 8 and 5% write drop everywhere."""
import os
import subprocess
import time

import pytest

from conftest import ROOT

SERVER = os.path.join(ROOT, "p1_amd", "p1server")
CLIENT = os.path.join(ROOT, "p1_amd", "p1client")
MINER = os.path.join(ROOT, "p1_amd", "p1miner")
FAKE = os.path.join(ROOT, "tools", "lsp_fake_miner")


class System:
    """One server + miners; every process is ours and is killed by PID."""

    def __init__(self, args=(), env=None):
        self.env = dict(os.environ, **(env or {}))
        self.procs = []
        self.server = subprocess.Popen([SERVER] + list(args) + ["lsp", "0"], stdout=subprocess.PIPE, text=True,
                                       env=self.env)
        self.procs.append(self.server)
        line = self.server.stdout.readline()  # server.go:79
        assert line.startswith("Server listening on port"), line
        self.port = int(line.split()[-1])
        self.hostport = f"127.0.0.1:{self.port}"

    def miner(self, cmd, env=None):
        argv = [self.hostport if c == "{hp}" else c for c in cmd]
        p = subprocess.Popen(argv, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                             env=dict(self.env, **(env or {})))
        self.procs.append(p)
        return p

    def client(self, msg, max_nonce, args=(), timeout=120, env=None):
        return subprocess.run([CLIENT, self.hostport, msg, str(max_nonce)] + list(args), capture_output=True,
                              text=True, timeout=timeout, env=dict(self.env, **(env or {})))

    def close(self):
        for p in self.procs:
            if p.poll() is None:
                p.kill()
            p.wait()


@pytest.fixture
def system():
    made = []

    def make(*a, **k):
        s = System(*a, **k)
        made.append(s)
        return s

    yield make
    for s in made:
        s.close()


def fake(args=()):
    return [FAKE, "{hp}"] + list(args)


def test_config1_client_server_one_cpu_miner(system, oracle_mod):
    # configs[0]: client 'bradfitz' maxNonce 9999 via server + 1 CPU miner
    s = system()
    s.miner(fake())
    r = s.client("bradfitz", 9999)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == "Result 1419516646206828 9898"


def test_split_over_miners_matches_oracle(system, oracle_mod):
    s = system(["--chunk", "1777"])
    for _ in range(4):
        s.miner(fake())
    for msg, mx in [("bradfitz", 99999), ("msg", 2), ("héllo wörld", 20000), ("", 0)]:
        r = s.client(msg, mx)
        h, n = oracle_mod.scan(msg, 0, mx, threads=4)
        assert r.stdout.strip() == f"Result {h} {n}", (msg, r.stdout, r.stderr)


def test_concurrent_clients(system, oracle_mod):
    s = system(["--chunk", "500"])
    for _ in range(3):
        s.miner(fake())
    jobs = [("a", 7000), ("bb", 3000), ("bradfitz", 9999), ("x" * 70, 5000)]
    procs = [subprocess.Popen([CLIENT, s.hostport, m, str(mx)], stdout=subprocess.PIPE, text=True)
             for m, mx in jobs]
    for (m, mx), p in zip(jobs, procs):
        out, _ = p.communicate(timeout=120)
        h, n = oracle_mod.scan(m, 0, mx, threads=4)
        assert out.strip() == f"Result {h} {n}", m


def test_write_drop_everywhere_small_epochs(system, oracle_mod):
    # 20% of every write lost in every process (lspnet.SetWriteDropPercent), window 4
    env = {"P1LSP_WRITE_DROP": "20"}
    prm = ["--epoch-millis", "50", "--epoch-limit", "20", "--window", "4"]
    s = system(["--chunk", "3000"] + prm, env=env)
    for _ in range(3):
        s.miner(fake(prm), env=env)
    r = s.client("bradfitz", 49999, args=prm, env=env)
    h, n = oracle_mod.scan("bradfitz", 0, 49999, threads=4)
    assert r.stdout.strip() == f"Result {h} {n}", r.stdout + r.stderr


def test_lost_miner_chunk_is_reassigned(system, oracle_mod):
    prm = ["--epoch-millis", "100", "--epoch-limit", "5"]
    s = system(["--chunk", "2000"] + prm)
    s.miner(fake(prm), env={"FAKE_DIE_AFTER": "2"})  # vanishes holding its 3rd chunk
    s.miner(fake(prm))
    r = s.client("bradfitz", 29999, args=prm)
    h, n = oracle_mod.scan("bradfitz", 0, 29999, threads=4)
    assert r.stdout.strip() == f"Result {h} {n}", r.stdout + r.stderr


def test_lost_client_does_not_block_others(system, oracle_mod):
    prm = ["--epoch-millis", "100", "--epoch-limit", "5"]
    s = system(["--chunk", "1000"] + prm)
    s.miner(fake(prm))
    # a client that vanishes right after sending a big request
    p = subprocess.Popen([CLIENT, s.hostport, "gone", str(10**7)] + prm, stdout=subprocess.DEVNULL)
    time.sleep(0.3)
    p.kill()
    p.wait()
    r = s.client("bradfitz", 9999, args=prm)
    assert r.stdout.strip() == "Result 1419516646206828 9898"


def test_client_reports_disconnected_when_server_dies(system):
    prm = ["--epoch-millis", "100", "--epoch-limit", "5"]
    s = system(prm)  # no miner: the request waits forever
    p = subprocess.Popen([CLIENT, s.hostport, "bradfitz", "9999"] + prm, stdout=subprocess.PIPE, text=True)
    time.sleep(0.3)
    s.server.kill()
    out, _ = p.communicate(timeout=60)
    assert out.strip() == "Disconnected"  # client.go:63-66
    assert p.returncode == 1


def test_client_fails_to_connect_without_server():
    r = subprocess.run([CLIENT, "127.0.0.1:9", "bradfitz", "9", "--epoch-millis", "50", "--epoch-limit", "3"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and r.stdout.startswith("Failed to connect to server")


def test_bad_arguments():
    r = subprocess.run([CLIENT, "127.0.0.1:9", "bradfitz", "x9"], capture_output=True, text=True, timeout=60)
    assert r.stdout.strip() == "x9 is not a number."
    r = subprocess.run([SERVER, "lsp", "abc"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Port must be a number" in r.stdout


@pytest.mark.gpu
def test_config5_over_lsp_8_gpu_miners_window8_drop5(system, oracle_mod):
    """configs[4]: the server splits [0, 2^36) into 2^32-nonce chunks over 8
    GPU miner processes (all on GPU 0 here), LSP window 8, 5% of every write
    dropped in every process.  Checked by size-independent properties: the
    nonce re-hashes to the hash on the oracle and equals the min of two
    independently scanned halves (through the library, one GPU)."""
    env = {"P1LSP_WRITE_DROP": "5"}
    prm = ["--window", "8"]
    s = system(["--chunk", str(1 << 32), "--exit-after", "1"] + prm, env=env)
    for _ in range(8):
        s.miner([MINER, "lsp", "{hp}", "--device", "0"] + prm, env=env)
    hi = (1 << 36) - 1
    t0 = time.time()
    r = s.client("bradfitz", hi, args=prm, timeout=600, env=env)
    wall = time.time() - t0
    assert r.returncode == 0, r.stdout + r.stderr
    word, h, n = r.stdout.split()
    h, n = int(h), int(n)
    assert word == "Result" and oracle_mod.hash("bradfitz", n) == h
    import p1_amd

    p1_amd.init_devices([0])
    a = p1_amd.scan("bradfitz", 0, (1 << 35) - 1)
    b = p1_amd.scan("bradfitz", 1 << 35, hi)
    assert min(a, b) == (h, n)
    print(f"configs[4] over LSP: 2^36 nonces, 8 GPU miners, window 8, 5% drop: {wall:.2f} s wall")
