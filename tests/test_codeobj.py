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


def test_shipped_build_uses_priorities_not_parity(codeobj):
    """Round 5: under per-run wave priorities the 4 (mod 8) parity rule of
    r01 no longer pays (r05aa A/B: its s_nops cost 0.3-1%), so the shipped
    post-pass runs the schedule and the priorities without it; the parity
    pass stays an option (DESIGN.md 4 "Dual issue")."""
    mk = open(os.path.join(ROOT, "Makefile")).read()
    line = next(ln for ln in mk.split("\n") if ln.startswith("ISAPOST ?="))
    assert "--pair-sched=0" in line and "--prio=0,1" in line and "--loop-parity" not in line, line
    assert "--no-e64" in line, line
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_parity.py"), codeobj],
                       capture_output=True, text=True, check=True)
    import json

    d = json.loads(r.stdout)
    assert d["loops"] >= 32, d


def test_scan_loops_keep_compiler_encodings(codeobj):
    """Round 5 (r05ad A/B: c3 +2.9%, c4 +0.3%): under per-run priorities the
    post-pass no longer widens full-rate VOP2 ops to VOP3 (r01's reason, the
    4 (mod 8) parity, is retired), so LLVM's 4-byte forms ship."""
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", codeobj], capture_output=True, text=True,
                         check=True).stdout
    n_e32 = len(re.findall(r"\bv_(add_u32|lshrrev_b32|xor_b32)_e32\b", dis))
    n_e64 = len(re.findall(r"\bv_(add_u32|lshrrev_b32|xor_b32)_e64\b", dis))
    assert n_e32 > 10000 and n_e64 < n_e32, (n_e32, n_e64)


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


def test_ab_nop_waits_before_full_rate_after_half_rate(tmp_path):
    """--ab-nop=3: one s_nop 3 before each full-rate VALU op that directly
    follows a half-rate one inside a loop, the 4 (mod 8) parity kept."""
    src, dst, obj = tmp_path / "a.s", tmp_path / "b.s", tmp_path / "b.o"
    src.write_text(SNIPPET)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_post.py"), str(src), str(dst),
                    "--align-loops=3", "--loop-offset=4", "--ab-nop=3", "--loop-parity"], check=True, capture_output=True)
    body = [ln.strip() for ln in dst.read_text().split("\n")]
    body = body[next(k for k, ln in enumerate(body) if ln.startswith(".LBB0_1:")):]
    for i in (k for k, ln in enumerate(body) if ln.startswith("v_alignbit_b32")):
        nxt = next(ln for ln in body[i + 1:] if ln.startswith("v_"))
        assert body[i + 1] == "s_nop 3" and isa_post.issue_class(nxt) == "B", body
    # add3 after the scalar s_add: no wait needed there, none inserted
    j = next(k for k, ln in enumerate(body) if ln.startswith("v_add3_u32"))
    assert not body[j - 1].startswith("s_nop 3")
    subprocess.run([f"{LLVM}/llvm-mc", "-arch=amdgcn", "-mcpu=gfx950", "-filetype=obj", "-o", str(obj), str(dst)],
                   check=True)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", str(obj)], capture_output=True, text=True,
                         check=True).stdout
    addr = [(int(m.group(2), 16), len(m.group(3).split()), m.group(1))
            for m in re.finditer(r"^\s+(\w+).*//\s*([0-9A-F]+):\s*((?:[0-9A-F]{8}\s*)+)$", dis, re.M)]
    assert all(a % 8 == 4 for a, n, op in addr if n == 2 and op.startswith("v_")), addr


def test_prio_switches_priority_per_run(tmp_path):
    """--prio=0,1: s_setprio 1 before the first half-rate op of every run,
    s_setprio 0 before the first full-rate op of every run, in loop bodies."""
    src, dst = tmp_path / "a.s", tmp_path / "b.s"
    src.write_text(SNIPPET)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_post.py"), str(src), str(dst),
                    "--align-loops=3", "--loop-offset=4", "--pair-sched=0", "--prio=0,1", "--loop-parity"],
                   check=True, capture_output=True)
    body = [ln.strip() for ln in dst.read_text().split("\n")]
    body = body[next(k for k, ln in enumerate(body) if ln.startswith(".LBB0_1:")):]
    prio, last = None, None
    for t in body:
        if t.startswith("s_setprio"):
            prio = int(t.split()[1])
        c = isa_post.issue_class(t) if t.startswith("v_") else None
        if c and c != last:
            assert prio == (1 if c == "A" else 0), (t, body)
        last = c or last
    assert sum(1 for t in body if t.startswith("s_setprio")) >= 2


def test_issue_classes():
    assert isa_post.issue_class("v_alignbit_b32 v1, v2, v2, 7") == "A"
    assert isa_post.issue_class("v_add3_u32 v1, v2, v3, v4") == "A"
    assert isa_post.issue_class("v_add_u32_e64 v42, s72, v35") == "A"  # VOP3 with an SGPR source (dual kind k)
    assert isa_post.issue_class("v_add_u32_e64 v42, v7, v35") == "B"
    assert isa_post.issue_class("v_bitop3_b32 v5, v1, v2, v3 bitop3:0x96") == "B"
    assert isa_post.issue_class("v_add_u32_e32 v1, s5, v2") == "B"
    assert isa_post.issue_class("s_nop 0") == "S"


# ---------------------------------------------------------------------------
# the roofline (0.649 on c4) sits at the floor of the
# loop mix, so a toolchain or post-pass change that lengthens the per-nonce
# loops is the only way left to lose it.  These counts are read off the
# shipped code object on the CPU and compared with the per-variant report
# (profiles/r03f_variant_report.jsonl, tools/variant_report.py: each variant
# built alone through the same pipeline).  The full kernel's register
# allocation moves a loop by up to 3 instructions either way against its
# single-variant build, hence the tolerance (3 VALU = 0.25% of a loop).
# ---------------------------------------------------------------------------
VARIANT_REPORT = os.path.join(ROOT, "profiles", "r03f_variant_report.jsonl")
# (FV, MODE, TRAIL): (half-rate A, full-rate B) VALU per nonce in its loop,
# for the decades that carry the bench workloads (bench.fast_variant)
PINNED_LOOPS = {
    (4, 6, False): (697, 500),   # c2 d = 10 (77% of configs[1]), c4 d = 10
    (3, 3, False): (697, 500),   # c2 d = 9 (21%)
    (4, 4, False): (684, 489),   # c4 d = 12 (64% of configs[3])
    (4, 1, False): (699, 503),   # c4 d = 11 (33%)
    (0, 5, False): (508, 381),   # c3 MODE 5, d = 9..11 (99% of configs[2])
    (15, 7, False): (505, 384),  # c3 MODE 7, d = 8
}
LOOP_TOL = 3


@pytest.fixture(scope="module")
def shipped_loops(codeobj):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import variant_report as vr

    ins, inner, _ = vr.loops_of(codeobj)
    per_nonce = [vr.mix(ins, *lp) for lp in inner]
    return [m for m in per_nonce if m["valu"] > 500]  # one nonce per iteration (the rest: setup, reduce)


def test_pinned_loop_counts_match_the_variant_report():
    """The constants above are the committed report's own numbers."""
    import json

    rows = {}
    for ln in open(VARIANT_REPORT):
        d = json.loads(ln)
        rows[tuple(d["variant"])] = (d["loop"]["half_rate_A"], d["loop"]["full_rate_B"])
    for v, ab in PINNED_LOOPS.items():
        assert rows[v] == ab, (v, rows[v], ab)
    sys.path.insert(0, ROOT)
    import bench

    # ... and they are the variants the bench workloads' big decades run
    assert bench.fast_variant(8, 10) == (4, 6, False) and bench.fast_variant(8, 9) == (3, 3, False)
    assert bench.fast_variant(8, 12) == (4, 4, False) and bench.fast_variant(8, 11) == (4, 1, False)
    assert bench.fast_variant(120, 10) == (0, 5, False) and bench.fast_variant(120, 8) == (15, 7, False)


def test_shipped_hot_loops_are_no_longer_than_pinned(shipped_loops):
    """Every pinned variant's loop is present in the shipped k_scan with its
    half-rate and full-rate counts within LOOP_TOL, and every per-nonce loop
    is free of memory instructions (no scratch spill reload per nonce)."""
    assert len(shipped_loops) == 63, len(shipped_loops)  # one per fast variant (fast_variants.inc)
    sigs = [(m["half_rate_A"], m["full_rate_B"]) for m in shipped_loops]
    for v, (a, b) in PINNED_LOOPS.items():
        near = [(x, y) for x, y in sigs if abs(x - a) <= LOOP_TOL and abs(y - b) <= LOOP_TOL]
        assert near, (v, (a, b), sorted(sigs))
        assert min(x + y for x, y in near) <= a + b + LOOP_TOL, (v, near)
    assert all(m["other"] == 0 for m in shipped_loops), [m for m in shipped_loops if m["other"]]


def test_shipped_hot_loops_switch_priority_per_run(codeobj):
    """Round 5: in every per-nonce loop each run of half-rate VALU ops starts
    with s_setprio 1 and each run of full-rate ones with s_setprio 0 (the
    dual-issue rule, DESIGN.md 4 "Dual issue": a half-rate op issues only as
    the first of a slot, beside a full-rate op of a lower-priority wave);
    losing it costs ~25%."""
    import variant_report as vr

    ins, inner, _ = vr.loops_of(codeobj)
    checked = 0
    for lo, hi in inner:
        body = [t for a, sz, t in ins if lo <= a <= hi]
        if sum(1 for t in body if t.startswith("v_")) <= 500:
            continue
        checked += 1
        last, prio, runs = None, None, 0
        for t in body:
            if t.startswith("s_setprio"):
                prio = int(t.split()[1], 0)
                continue
            if t.startswith(("v_cndmask", "v_cmp")):
                continue  # the argmin tail (the parity pass may widen it after --prio ran)
            op = t.split()[0]
            if op.endswith("_e64") and not op.startswith(isa_post.E32_OPS):
                t = t.replace("_e64", "_e32", 1)  # widened by the parity pass after --prio classified it
            c = isa_post.issue_class(t)
            if c in "AB":
                if c != last:
                    runs += 1
                    assert prio == (1 if c == "A" else 0), (hex(lo), t, prio)
                last = c
        assert runs > 100, (hex(lo), runs)
    assert checked == 63, checked


def test_k_scan_registers_keep_four_waves(codeobj):
    """<= 128 VGPRs (4 waves/SIMD, DESIGN.md 4 "Occupancy budget") and <= 106
    SGPRs (the 64 round constants in SGPRs)."""
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", codeobj], capture_output=True, text=True,
                           check=True).stdout
    blk = notes[notes.index(".name:           k_scan\n"):]
    get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))  # noqa: E731
    assert get("vgpr_count") <= 128 and get("sgpr_count") <= 106, (get("vgpr_count"), get("sgpr_count"))


def test_branches_fit_after_the_post_pass_growth(codeobj):
    """Makefile -amdgpu-s-branch-bits=15: the post-pass inserts its
    s_setprio and loop padding after LLVM relaxed the branches, so LLVM is
    told branches reach +-2^14 dwords of the real +-2^15.  The shipped
    object's largest displacement stays inside the real range with room to
    spare; the per-nonce loops contain no long (s_setpc) branch."""
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", codeobj], capture_output=True, text=True,
                         check=True).stdout
    offs = []
    for m in re.finditer(r"\bs_(?:c)?branch\w*\s+(\d+)\s+//", dis):
        v = int(m.group(1))
        offs.append(v - 65536 if v >= 32768 else v)
    assert len(offs) > 500
    assert max(abs(v) for v in offs) < 1 << 15
    assert dis.count("s_setprio") > 20000


def test_assembler_rejects_a_branch_out_of_range(tmp_path):
    """Why the branch margin is safe by construction: a short branch the
    growth pushed out of range fails the build's assembly step (the
    Makefile's clang -cc1as) instead of producing a wrong target."""
    src = tmp_path / "far.s"
    src.write_text(".text\nf:\n s_branch .Lend\n" + " s_nop 0\n" * 33000 + ".Lend:\n s_endpgm\n")
    r = subprocess.run([f"{LLVM}/clang", "-cc1as", "-triple", "amdgcn-amd-amdhsa", "-filetype", "obj", "-target-cpu",
                        "gfx950", "-o", str(tmp_path / "far.o"), str(src)], capture_output=True, text=True)
    assert r.returncode != 0 and "branch size exceeds simm16" in r.stderr, r.stderr[-500:]


def test_codeobj_sha256_is_the_embedded_object():
    """p1_amd.codeobj_sha256 (what bench.py reports and matches profiles
    by) hashes exactly the code object embedded in the library, which is
    build/p1hip_kernels.hsaco when the build tree is present."""
    import hashlib

    sys.path.insert(0, ROOT)
    import p1_amd

    blob = p1_amd.codeobj_bytes()
    assert blob[:4] == b"\x7fELF" and blob == embedded_code_object()
    assert p1_amd.codeobj_sha256() == hashlib.sha256(blob).hexdigest()
    hsaco = os.path.join(ROOT, "build", "p1hip_kernels.hsaco")
    if os.path.exists(hsaco):
        assert open(hsaco, "rb").read() == blob
