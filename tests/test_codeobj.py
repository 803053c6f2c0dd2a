"""The gfx950 code object embedded in libp1hip.so and the assembly post-pass
that builds it (tools/isa_post.py).  CPU only: disassembly, no execution."""
import os
import re
import struct
import subprocess
import sys
import tempfile

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_post  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"


def embedded_code_object():
    """The AMDGPU ELF inside libp1hip.so's .rodata (p1hip_kernels_blob.S)."""
    blob = open(os.path.join(ROOT, "p1_amd", "libp1hip.so"), "rb").read()
    at = 1
    while True:
        at = blob.find(b"\x7fELF", at)
        assert at > 0, "no embedded code object"
        e_machine = struct.unpack_from("<H", blob, at + 18)[0]
        if e_machine == 224:  # EM_AMDGPU
            break
        at += 4
    e_shoff, = struct.unpack_from("<Q", blob, at + 0x28)
    e_shentsize, e_shnum = struct.unpack_from("<HH", blob, at + 0x3A)
    return blob[at:at + e_shoff + e_shentsize * e_shnum]


@pytest.fixture(scope="module")
def codeobj(tmp_path_factory):
    p = tmp_path_factory.mktemp("co") / "p1hip_kernels.hsaco"
    p.write_bytes(embedded_code_object())
    return str(p)


def test_code_object_is_gfx950_with_all_kernels(codeobj):
    hdr = subprocess.run([f"{LLVM}/llvm-readelf", "-h", "-s", codeobj], capture_output=True, text=True, check=True).stdout
    assert "EM_AMDGPU" in hdr and "gfx950" in hdr
    for k in ("k_scan", "k_reduce", "k_pairs"):
        assert re.search(rf"FUNC\s+GLOBAL\s+\w+\s+\d+\s+{k}$", hdr, re.M), k
        assert f"{k}.kd" in hdr


def test_hot_loops_keep_4_mod_8_parity(codeobj):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_parity.py"), codeobj],
                       capture_output=True, text=True, check=True)
    import json

    d = json.loads(r.stdout)
    assert d["loops"] >= 32 and d["frac"] > 0.99, d


def test_scan_loops_are_vop3_only(codeobj):
    """Inside the loops no full-rate op is left in its 4-byte VOP2 form."""
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", codeobj], capture_output=True, text=True,
                         check=True).stdout
    n_e32 = len(re.findall(r"\bv_(add_u32|lshrrev_b32|xor_b32)_e32\b", dis))
    n_e64 = len(re.findall(r"\bv_(add_u32|lshrrev_b32|xor_b32)_e64\b", dis))
    assert n_e64 > 10000 and n_e32 < n_e64 // 50, (n_e32, n_e64)


def test_widen_and_convertible():
    assert isa_post.widen("\tv_cndmask_b32_e32 v9, v9, v35, vcc") == "\tv_cndmask_b32_e64 v9, v9, v35, vcc"
    assert isa_post.widen("\tv_cmp_lt_u64_e32 vcc, v[34:35], v[8:9]") == "\tv_cmp_lt_u64_e64 vcc, v[34:35], v[8:9]"
    assert isa_post.widen("\tv_mov_b32_e32 v33, s68") == "\tv_mov_b32_e64 v33, s68"
    assert isa_post.widen("\tv_add_u32_e32 v1, 0x428a2f98, v2") is None  # literal: VOP3 cannot hold it
    assert isa_post.widen("\tv_add_u32_dpp v0, v1, v2 row_ror:4") is None
    assert isa_post.convertible("v1, s6, v34") and isa_post.convertible("v1, 3, v2")
    assert not isa_post.convertible("v1, 0xb5c0fbcf, v2")


SNIPPET = """\t.text
\t.p2align 8
f:
\ts_mov_b32 s0, 8
.LBB0_1:                                ; =>This Inner Loop Header: Depth=1
\tv_alignbit_b32 v1, v1, v1, 7
\tv_add_u32_e32 v2, v1, v2
\tv_alignbit_b32 v3, v2, v2, 13
\tv_mov_b32_e32 v4, s0
\tv_bitop3_b32 v5, v1, v2, v3 bitop3:0x96
\ts_add_i32 s0, s0, -1
\tv_add3_u32 v6, v5, v4, v3
\ts_cmp_eq_u32 s0, 0
\ts_cbranch_scc0 .LBB0_1
\ts_endpgm
"""


def test_post_pass_assembles_with_parity(tmp_path):
    src, dst, obj = tmp_path / "a.s", tmp_path / "b.s", tmp_path / "b.o"
    src.write_text(SNIPPET)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_post.py"), str(src), str(dst),
                    "--align-loops=3", "--loop-offset=4", "--loop-parity"], check=True, capture_output=True)
    out = dst.read_text()
    assert "v_add_u32_e64 v2, v1, v2" in out
    subprocess.run([f"{LLVM}/llvm-mc", "-arch=amdgcn", "-mcpu=gfx950", "-filetype=obj", "-o", str(obj), str(dst)],
                   check=True)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", str(obj)], capture_output=True, text=True,
                         check=True).stdout
    addr = [(int(m.group(2), 16), len(m.group(3).split()), m.group(1))
            for m in re.finditer(r"^\s+(\w+).*//\s*([0-9A-F]+):\s*((?:[0-9A-F]{8}\s*)+)$", dis, re.M)]
    loop = [a for a in addr if a[2] in ("v_alignbit_b32", "v_bitop3_b32", "v_add3_u32", "v_add_u32_e64")]
    assert len(loop) == 5 and all(a % 8 == 4 for a, n, _ in loop if n == 2), addr
