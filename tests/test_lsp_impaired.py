"""The bitcoin system over LSP through an impaired network: every datagram
between the server and its peers passes a UDP proxy that drops 10%,
duplicates 10% and delays each by 0-40 ms (so datagrams overtake each
other).  The reference's tests inject loss only (lspnet drop knobs); UDP
also reorders and duplicates, which the window, the in-order receiver and
the acks must absorb.  The clients must print the exact answers.  Runs the
ASan + UBSan builds (`make sanitize`) with no sanitizer report."""
import heapq
import os
import random
import select
import socket
import subprocess
import threading
import time

import pytest

from conftest import ROOT

SAN = os.path.join(ROOT, "build", "san", "asan")
SANCXX = "/opt/rocm/lib/llvm/bin/clang++"

pytestmark = pytest.mark.skipif(not os.path.exists(SANCXX), reason="ROCm clang (sanitizer runtimes) not present")


class ImpairedProxy(threading.Thread):
    """Listens on a port; each peer address gets its own upstream socket to
    the server (so the server sees one stable address per peer).  Both
    directions are dropped / duplicated / delayed."""

    def __init__(self, server_port, seed, drop=0.10, dup=0.10, max_delay=0.040):
        super().__init__(daemon=True)
        self.server = ("127.0.0.1", server_port)
        self.rnd = random.Random(seed)
        self.drop, self.dup, self.max_delay = drop, dup, max_delay
        self.front = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.front.bind(("127.0.0.1", 0))
        self.port = self.front.getsockname()[1]
        self.up = {}      # peer addr -> upstream socket
        self.down = {}    # upstream socket -> peer addr
        self.queue = []   # (due, seq, sock, data, addr)
        self.seq = 0
        self.stop = threading.Event()
        self.stats = {"in": 0, "dropped": 0, "duplicated": 0}

    def schedule(self, sock, data, addr):
        self.stats["in"] += 1
        if self.rnd.random() < self.drop:
            self.stats["dropped"] += 1
            return
        copies = 2 if self.rnd.random() < self.dup else 1
        self.stats["duplicated"] += copies - 1
        for _ in range(copies):
            self.seq += 1
            heapq.heappush(self.queue, (time.monotonic() + self.rnd.uniform(0, self.max_delay), self.seq, sock, data,
                                        addr))

    def run(self):
        while not self.stop.is_set():
            timeout = 0.005
            if self.queue:
                timeout = max(0.0, min(timeout, self.queue[0][0] - time.monotonic()))
            r, _, _ = select.select([self.front] + list(self.down), [], [], timeout)
            for s in r:
                try:
                    data, addr = s.recvfrom(65536)
                except OSError:
                    continue
                if s is self.front:
                    u = self.up.get(addr)
                    if u is None:
                        u = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
                        u.bind(("127.0.0.1", 0))
                        self.up[addr] = u
                        self.down[u] = addr
                    self.schedule(u, data, self.server)
                else:
                    self.schedule(self.front, data, self.down[s])
            now = time.monotonic()
            while self.queue and self.queue[0][0] <= now:
                _, _, sock, data, addr = heapq.heappop(self.queue)
                try:
                    sock.sendto(data, addr)
                except OSError:
                    pass


def test_system_through_reordering_duplicating_lossy_network(tmp_path, oracle_mod):
    subprocess.run(["make", "-s", "-j8", "-C", ROOT, "sanitize"], check=True, stdout=subprocess.DEVNULL)
    env = dict(os.environ,
               ASAN_OPTIONS=f"detect_leaks=1:log_path={tmp_path}/asan",
               UBSAN_OPTIONS=f"print_stacktrace=1:halt_on_error=1:log_path={tmp_path}/ubsan")
    prm = ["--epoch-millis", "60", "--epoch-limit", "30", "--window", "4", "--copies", "1"]
    procs = []
    proxy = None
    try:
        srv = subprocess.Popen([os.path.join(SAN, "p1server"), "--chunk", "1200"] + prm + ["lsp", "0"],
                               stdout=subprocess.PIPE, text=True, env=env)
        procs.append(srv)
        line = srv.stdout.readline()
        assert line.startswith("Server listening on port"), line
        proxy = ImpairedProxy(int(line.split()[-1]), seed=440)
        proxy.start()
        hp = f"127.0.0.1:{proxy.port}"
        for _ in range(3):
            procs.append(subprocess.Popen([os.path.join(SAN, "lsp_fake_miner"), hp] + prm, env=env,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        jobs = [("bradfitz", 19999), ("cmu440", 9000), ("héllo", 12000), ("", 5000)]
        clients = [subprocess.Popen([os.path.join(SAN, "p1client"), hp, m, str(mx)] + prm, stdout=subprocess.PIPE,
                                    stderr=subprocess.PIPE, text=True, env=env) for m, mx in jobs]
        for (m, mx), c in zip(jobs, clients):
            out, err = c.communicate(timeout=240)
            h, n = oracle_mod.scan(m, 0, mx, threads=4)
            assert out.strip() == f"Result {h} {n}", (m, out, err[-2000:], proxy.stats)
        st = proxy.stats
        assert st["dropped"] > 20 and st["duplicated"] > 20, st  # the impairments really happened
    finally:
        if proxy:
            proxy.stop.set()
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    reports = sorted(f for f in os.listdir(tmp_path) if f.split(".")[0] in ("asan", "ubsan"))
    assert not reports, "".join(open(os.path.join(tmp_path, f)).read()[:4000] for f in reports)
