"""The host programs under ASan + UBSan and TSan (CPU only).

`make sanitize` builds the LSP stack, the server, the client, the CPU test
double miner and the scheduler unit test with each sanitizer (ROCm's clang;
DESIGN.md §6 "Host code under sanitizers").  Here the reference LSP
scenarios run under the two builds (half under each) with the production
default of three copies per first Data transmission (lsp::DefaultAppCopies),
the scheduler unit test
under ASan, and a whole
server + miners + client system under loss under both; a run passes only
if it succeeds AND leaves no sanitizer report file.  tools/sanitize.sh
re-runs the full host-program test modules the same way."""
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

from conftest import ROOT

SAN = os.path.join(ROOT, "build", "san")
SANCXX = "/opt/rocm/lib/llvm/bin/clang++"

pytestmark = pytest.mark.skipif(not os.path.exists(SANCXX), reason="ROCm clang (sanitizer runtimes) not present")


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-j8", "-C", ROOT, "sanitize"], check=True, stdout=subprocess.DEVNULL)


def san_env(kind, logs):
    return dict(os.environ,
                ASAN_OPTIONS=f"detect_leaks=1:log_path={logs}/asan",
                UBSAN_OPTIONS=f"print_stacktrace=1:halt_on_error=1:log_path={logs}/ubsan",
                TSAN_OPTIONS=f"halt_on_error=0:log_path={logs}/tsan")


def reports(logs):
    out = []
    for f in sorted(os.listdir(logs)):
        if f.split(".")[0] in ("asan", "ubsan", "tsan"):
            with open(os.path.join(logs, f)) as fh:
                out.append(f + ":\n" + fh.read()[:4000])
    return out


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_lsp_scenarios_under_sanitizer(kind, tmp_path):
    drv = os.path.join(SAN, kind, "lsp_scenarios")
    env = san_env(kind, tmp_path)
    names = subprocess.run([drv, "--list"], capture_output=True, text=True, check=True, env=env).stdout.split()
    assert len(names) == 48
    # every other scenario keeps the CPU suite short; tools/sanitize.sh runs
    # all 48 at 1 and 2 copies under both sanitizers; here the programs'
    # default, lsp::DefaultAppCopies = 3
    names = names[::2] if kind == "tsan" else names[1::2]

    def run(name):
        r = subprocess.run([drv, "--copies", "3", name], capture_output=True, text=True, timeout=240, env=env)
        return name, r.returncode, r.stdout + r.stderr

    with ThreadPoolExecutor(max_workers=6) as ex:
        results = list(ex.map(run, names))
    failed = [(n, rc, out[-2000:]) for n, rc, out in results if rc != 0 or not out.startswith(f"{n} PASS")]
    assert not failed, failed
    assert not reports(tmp_path), reports(tmp_path)


def test_scheduler_under_asan(tmp_path):
    r = subprocess.run([os.path.join(SAN, "asan", "sched_test")], capture_output=True, text=True, timeout=120,
                       env=san_env("asan", tmp_path))
    assert r.returncode == 0 and r.stdout.strip() == "sched_test: ok", r.stdout + r.stderr
    assert not reports(tmp_path), reports(tmp_path)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_system_under_loss_under_sanitizer(kind, tmp_path, oracle_mod):
    """p1server lsp + 3 test-double miners + 2 concurrent clients, 20% of
    every write dropped everywhere, small epochs, window 4; one miner dies
    holding a chunk (its chunk must be reassigned)."""
    d = os.path.join(SAN, kind)
    env = dict(san_env(kind, tmp_path), P1LSP_WRITE_DROP="20")
    prm = ["--epoch-millis", "50", "--epoch-limit", "20", "--window", "4"]
    procs = []
    try:
        srv = subprocess.Popen([os.path.join(d, "p1server"), "--chunk", "2000"] + prm + ["lsp", "0"],
                               stdout=subprocess.PIPE, text=True, env=env)
        procs.append(srv)
        line = srv.stdout.readline()
        assert line.startswith("Server listening on port"), line
        hp = f"127.0.0.1:{int(line.split()[-1])}"
        for i in range(3):
            menv = dict(env, FAKE_DIE_AFTER="2") if i == 0 else env
            procs.append(subprocess.Popen([os.path.join(d, "lsp_fake_miner"), hp] + prm, env=menv,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        jobs = [("bradfitz", 19999), ("héllo", 7000)]
        clients = [subprocess.Popen([os.path.join(d, "p1client"), hp, m, str(mx)] + prm, stdout=subprocess.PIPE,
                                    stderr=subprocess.PIPE, text=True, env=env) for m, mx in jobs]
        for (m, mx), c in zip(jobs, clients):
            out, err = c.communicate(timeout=240)
            h, n = oracle_mod.scan(m, 0, mx, threads=4)
            assert out.strip() == f"Result {h} {n}", (m, out, err[-2000:])
    finally:
        # the server and miners serve until killed, so only the clients (and
        # lsp_scenarios above) reach LeakSanitizer's exit-time check; every
        # other report is written when the error happens, before this
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    assert not reports(tmp_path), reports(tmp_path)
