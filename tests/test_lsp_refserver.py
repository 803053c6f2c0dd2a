"""Our LSP clients against a server that behaves like the REFERENCE's on the
connect path.

The reference server has no per-address lookup: read() hands every Connect
datagram to chanNewConn (lsp/server_impl.go:198-200), and the state machine
makes each one a new connection -- a fresh connId, window, sorter and epoch
goroutine, and an Ack(connId, 0) (server_impl.go:117-137).  A client that
sent its Connect three times would therefore own three connections there,
two of them phantoms.  `RefShapedServer` below restates exactly that connect
path (plus Data -> Ack, server_impl.go:163-167) in a few lines of Python, and
answers the bitcoin messages itself (a Request with the oracle's Result, a
miner's Join with one Request), so each program also completes a real
exchange over it.

CPU tests: p1client and tools/lsp_fake_miner (the miner loop of p1miner with
the oracle instead of the GPU; same lsp::Client code).  GPU test: p1miner.
"""
import base64
import json
import os
import socket
import subprocess
import threading
import time

import pytest

from conftest import ROOT, host_bin

CLIENT = host_bin(os.path.join(ROOT, "p1_amd", "p1client"))
MINER = host_bin(os.path.join(ROOT, "p1_amd", "p1miner"))
FAKE = host_bin(os.path.join(ROOT, "tools", "lsp_fake_miner"))

MSG_CONNECT, MSG_DATA, MSG_ACK = 0, 1, 2           # lsp/message.go:11-13
JOIN, REQUEST, RESULT = 0, 1, 2                    # bitcoin/message.go:8-10


def _lsp(t, conn, seq, payload=None):
    # encoding/json of lsp.Message: []byte payload as base64, nil as null
    return json.dumps({"Type": t, "ConnID": conn, "SeqNum": seq, "Size": len(payload) if payload else 0,
                       "Payload": base64.b64encode(payload).decode() if payload else None}).encode()


def _btc(t, data="", lower=0, upper=0, h=0, n=0):
    return json.dumps({"Type": t, "Data": data, "Lower": lower, "Upper": upper, "Hash": h, "Nonce": n}).encode()


class RefShapedServer:
    """The reference server's connect path: one new connection per Connect
    datagram, ids from 1 (server_impl.go:69-75,117-137,198-200)."""

    def __init__(self, oracle, request=("bradfitz", 0, 999)):
        self.oracle, self.request = oracle, request
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.settimeout(0.1)
        self.port = self.sock.getsockname()[1]
        self.conns = {}          # connId -> client address
        self.connects = 0        # Connect datagrams read
        self.results = []        # (connId, hash, nonce) from miners
        self.next_seq = {}       # connId -> next outgoing data seq (InitSeqNum + 1)
        self.seen = set()        # (connId, seq) delivered once (the sorter)
        self.stop = False
        self.th = threading.Thread(target=self._run, daemon=True)
        self.th.start()

    def _send_data(self, conn, payload):
        seq = self.next_seq[conn]
        self.next_seq[conn] += 1
        self.sock.sendto(_lsp(MSG_DATA, conn, seq, payload), self.conns[conn])

    def _run(self):
        while not self.stop:
            try:
                buf, addr = self.sock.recvfrom(4096)
            except socket.timeout:
                continue
            m = json.loads(buf)
            if m["Type"] == MSG_CONNECT:
                # chanNewConn <- cAddr: no lookup of cAddr, always a new id
                self.connects += 1
                cid = len(self.conns) + 1
                self.conns[cid] = addr
                self.next_seq[cid] = 1
                self.sock.sendto(_lsp(MSG_ACK, cid, 0), addr)
                continue
            cid = m["ConnID"]
            if cid not in self.conns or m["Type"] != MSG_DATA:
                continue
            self.sock.sendto(_lsp(MSG_ACK, cid, m["SeqNum"]), addr)  # server_impl.go:165-167
            if (cid, m["SeqNum"]) in self.seen:
                continue
            self.seen.add((cid, m["SeqNum"]))
            b = json.loads(base64.b64decode(m["Payload"]))
            if b["Type"] == REQUEST:  # a client: answer with the oracle
                h, n = self.oracle.scan(b["Data"], b["Lower"], b["Upper"])
                self._send_data(cid, _btc(RESULT, h=h, n=n))
            elif b["Type"] == JOIN:  # a miner: hand it one request
                self._send_data(cid, _btc(REQUEST, *self.request))
            elif b["Type"] == RESULT:
                self.results.append((cid, b["Hash"], b["Nonce"]))

    def close(self):
        self.stop = True
        self.th.join()
        self.sock.close()


@pytest.fixture
def refserver(oracle_mod):
    made = []

    def make(**k):
        s = RefShapedServer(oracle_mod, **k)
        made.append(s)
        return s

    yield make
    for s in made:
        s.close()


def _env():
    env = dict(os.environ)
    for k in list(env):
        if k.startswith("P1LSP_"):
            del env[k]
    return env


def test_client_opens_one_connection_on_a_reference_server(refserver, oracle_mod):
    """configs[0]'s client at default settings (3 copies of every Data
    message) opens exactly one connection, and gets its Result."""
    srv = refserver()
    r = subprocess.run([CLIENT, f"127.0.0.1:{srv.port}", "bradfitz", "9999", "--epoch-millis", "300"],
                       capture_output=True, text=True, timeout=60, env=_env())
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == "Result 1419516646206828 9898"
    assert srv.connects == 1 and len(srv.conns) == 1


def test_miner_opens_one_connection_on_a_reference_server(refserver, oracle_mod):
    """The miner's join + one Request -> Result exchange (miner.go:13-73) at
    default settings: one connection on the reference-shaped server."""
    srv = refserver()
    p = subprocess.Popen([FAKE, f"127.0.0.1:{srv.port}", "--epoch-millis", "300"], stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL, env=_env())
    try:
        t0 = time.time()
        while not srv.results and time.time() - t0 < 30:
            time.sleep(0.05)
        time.sleep(0.9)  # three more epochs: an extra Connect would show now
    finally:
        p.kill()
        p.wait()
    want = oracle_mod.scan("bradfitz", 0, 999)
    assert srv.results == [(1, want[0], want[1])]
    assert srv.connects == 1 and len(srv.conns) == 1


def test_connect_copies_above_one_open_phantoms_there(refserver):
    """Why Params::ConnectCopies defaults to 1: with 3 Connect copies the
    reference-shaped server opens 3 connections for one client (our own
    server answers all three with one id, lsp.cpp ServerImpl::on_msg)."""
    srv = refserver()
    r = subprocess.run([CLIENT, f"127.0.0.1:{srv.port}", "bradfitz", "99", "--epoch-millis", "300",
                        "--connect-copies", "3"], capture_output=True, text=True, timeout=60, env=_env())
    assert r.returncode == 0, r.stdout + r.stderr
    assert srv.connects == 3 and len(srv.conns) == 3


@pytest.mark.gpu
def test_gpu_miner_opens_one_connection_on_a_reference_server(refserver, oracle_mod):
    """p1miner itself (GPU-backed scan) against the reference-shaped server."""
    srv = refserver(request=("bradfitz", 0, 99999))
    p = subprocess.Popen([MINER, "lsp", f"127.0.0.1:{srv.port}", "--device", "0", "--epoch-millis", "300"],
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=_env())
    try:
        t0 = time.time()
        while not srv.results and time.time() - t0 < 60:
            time.sleep(0.05)
        time.sleep(0.9)
    finally:
        p.kill()
        p.wait()
    want = oracle_mod.scan("bradfitz", 0, 99999)
    assert srv.results == [(1, want[0], want[1])]
    assert srv.connects == 1 and len(srv.conns) == 1
