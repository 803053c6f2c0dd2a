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
