"""The C ABI from C: include/p1hip.h compiles as strict C99 and a C program
links libp1hip.so (what a cgo bridge does)."""
import os
import subprocess

import pytest

from conftest import ROOT


def _build(tmp_path):
    exe = tmp_path / "capi_smoke"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "capi_smoke.c"),
                    "-L", os.path.join(ROOT, "p1_amd"), "-lp1hip",
                    f"-Wl,-rpath,{os.path.join(ROOT, 'p1_amd')}", "-o", str(exe)], check=True)
    return str(exe)


def test_header_is_c99_and_links(tmp_path):
    exe = _build(tmp_path)
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", "0").split(",")[0])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    try:
        import torch

        has_gpu = torch.cuda.device_count() > 0
    except ImportError:
        has_gpu = False
    if has_gpu:
        assert r.returncode == 0 and r.stdout.strip() == "Result 1419516646206828 9898", r.stdout + r.stderr
    else:
        assert r.returncode == 0 and r.stdout.startswith("nodevice"), r.stdout + r.stderr


@pytest.mark.gpu
def test_c_client_on_gpu(tmp_path):
    exe = _build(tmp_path)
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", "0").split(",")[0])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip() == "Result 1419516646206828 9898"


def _build_chunkloop(tmp_path):
    exe = tmp_path / "capi_chunkloop"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "capi_chunkloop.c"),
                    "-L", os.path.join(ROOT, "p1_amd"), "-lp1hip", f"-Wl,-rpath,{os.path.join(ROOT, 'p1_amd')}",
                    "-L", os.path.join(ROOT, "oracle"), "-lp1oracle", f"-Wl,-rpath,{os.path.join(ROOT, 'oracle')}",
                    "-o", str(exe)], check=True)
    return str(exe)


def test_chunkloop_builds_and_reports_no_device(tmp_path):
    """INTEGRATION.md's chunk loop links as plain C; without a GPU the
    library answers rc -1 (no CPU fallback inside the library)."""
    exe = _build_chunkloop(tmp_path)
    try:
        import torch

        if torch.cuda.device_count() > 0:
            pytest.skip("GPU present: covered by test_chunkloop_on_gpu")
    except ImportError:
        pass
    r = subprocess.run([exe, "bradfitz", "0", "9999", "1000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("nodevice"), r.stdout + r.stderr


@pytest.mark.gpu
def test_chunkloop_on_gpu(tmp_path, oracle_mod):
    """The Go bridge's loop through the C ABI: chunked
    scans equal one scan; the rc != 0 branch (an invalid argument on every
    3rd chunk) falls back to the reference's CPU loop for that chunk and the
    result is unchanged (miner.go:49-71)."""
    exe = _build_chunkloop(tmp_path)
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", "0").split(",")[0])
    for msg, lo, hi, chunk in [("bradfitz", 0, 99999, 7919), ("msg", 0, 2, 1), ("x" * 70, 10**9 - 5000, 10**9 + 5000, 997)]:
        want = oracle_mod.scan(msg, lo, hi, threads=8)
        r = subprocess.run([exe, msg, str(lo), str(hi), str(chunk)], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        assert r.stdout.split()[:3] == ["Result", str(want[0]), str(want[1])], (msg, r.stdout)
        assert "cpu_chunks=0" in r.stdout
        r = subprocess.run([exe, msg, str(lo), str(hi), str(chunk), "3"], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        assert r.stdout.split()[:3] == ["Result", str(want[0]), str(want[1])], (msg, r.stdout)
        if (hi - lo + 1) // chunk >= 3:
            assert "cpu_chunks=0" not in r.stdout


def test_go_binding_plan_shards_edges(tmp_path):
    """INTEGRATION.md's gpu.PlanShards through the C ABI as the binding calls
    it: n = 0 and n < 0 return the library's
    P1HIP_ERR_ARGS with its message (the binding must not index &f[0]), and
    n >= 1 gives n in-order contiguous shards over [lower, upper]; lower >
    upper gives n empty shards.  Host only (no device)."""
    exe = tmp_path / "capi_plan_shards"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "capi_plan_shards.c"),
                    "-L", os.path.join(ROOT, "p1_amd"), "-lp1hip", f"-Wl,-rpath,{os.path.join(ROOT, 'p1_amd')}",
                    "-o", str(exe)], check=True)

    def run(*a):
        r = subprocess.run([str(exe)] + [str(x) for x in a], capture_output=True, text=True, timeout=60)
        return r.returncode, r.stdout.splitlines()

    for n in (0, -1, -(2 ** 31)):
        rc, out = run("bradfitz", 0, 9999, n)
        assert rc == 0 and out[0].startswith("rc -4 ") and "n <= 0" in out[0], out
    rc, out = run("", 0, 9999, 0)  # empty message: NULL msg pointer with length 0 is valid
    assert rc == 0 and out[0].startswith("rc -4 "), out
    for msg, lo, hi, n in [("bradfitz", 0, (1 << 38) - 1, 8), ("bradfitz", 0, 9999, 1), ("x" * 70, 10, 12, 8),
                           ("", 0, 0, 3), ("bradfitz", 2 ** 64 - 100, 2 ** 64 - 1, 4)]:
        rc, out = run(msg, lo, hi, n)
        assert rc == 0 and out[0] == "ok" and len(out) == n + 1, (msg, lo, hi, n, out)
    rc, out = run("bradfitz", 7, 3, 5)  # lower > upper: n empty shards, rc 0
    assert rc == 0 and out[0] == "ok" and all(line.endswith(" 0") for line in out[1:]) and len(out) == 6


SAN_DIR = os.path.join(ROOT, "tools", "san")
SAN_STRESS = os.path.join(SAN_DIR, "capi_san_stress")
# what `make sanitize-lib` produces (Makefile SANLIB); all of it is rebuilt
# from this tree's sources by the test itself, never taken as found
SAN_OUTPUTS = ["p1hip_host.o", "libp1hip.so", "capi_san_stress", "p1miner"]


def build_sanitize_lib():
    """Delete every ASan artefact and rebuild it from the checked-out
    sources (a binary pushed from elsewhere, or one
    older than the sources, must never be what the test runs).  Host code
    only, ~25 s; the kernels are the shipped code object
    (build/p1hip_kernels_blob.o, which `make all` made for libp1hip.so)."""
    for f in SAN_OUTPUTS:
        try:
            os.remove(os.path.join(SAN_DIR, f))
        except FileNotFoundError:
            pass
    jobs = str(min(16, os.cpu_count() or 1))
    r = subprocess.run(["make", "-s", "-C", ROOT, "-j", jobs, "sanitize-lib"], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert os.path.exists(SAN_STRESS)


@pytest.mark.gpu
def test_host_runtime_under_asan(tmp_path):
    """The library's host runtime built with ASan + UBSan on the host side
    (`make sanitize-lib`, rebuilt here from the tree's sources; the kernels
    are the shipped code object) drives real scans for 40 s: planner,
    argument errors, exact and property-checked random scans, 4 host threads
    at once, the argmin on crafted pairs, 3 logical devices with host
    combine, launch / table / span caps, an injected device failure and
    recovery, re-init cycles (tests/capi_san_stress.cpp).  Passes only with
    rc 0 and no report file."""
    build_sanitize_lib()
    env = dict(os.environ,
               ASAN_OPTIONS=f"detect_leaks=1:log_path={tmp_path}/asan",
               LSAN_OPTIONS=f"suppressions={os.path.join(ROOT, 'tests', 'lsan_rocm.supp')}:print_suppressions=0",
               UBSAN_OPTIONS=f"print_stacktrace=1:halt_on_error=1:log_path={tmp_path}/ubsan")
    for k in list(env):
        if k.startswith("P1HIP_"):
            del env[k]
    r = subprocess.run([SAN_STRESS, "40"], capture_output=True, text=True, timeout=110, env=env)
    reports = sorted(f for f in os.listdir(tmp_path) if f.split(".")[0] in ("asan", "ubsan"))
    text = "".join(open(os.path.join(tmp_path, f)).read()[:4000] for f in reports)
    print(r.stdout)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr + text
    assert not reports, text
