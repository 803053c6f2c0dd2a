"""tools/pair_sched.py: the post-RA reordering of loop segments for dual
issue keeps every register dependency and never moves an instruction across
a barrier.  CPU only."""
import json
import os
import random
import re
import subprocess
import sys
import tempfile

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_post  # noqa: E402
import pair_sched  # noqa: E402


def test_parse_defs_uses():
    d, u = pair_sched.parse("v_add3_u32 v47, v47, v48, s68")
    assert d == {"v47"} and u == {"v47", "v48", "s68", "exec"}
    d, u = pair_sched.parse("s_lshr_b32 s73, s72, 7")
    assert d == {"s73", "scc"} and u == {"s72"}
    d, u = pair_sched.parse("v_bitop3_b32 v55, v44, v38, v11 bitop3:0xca")
    assert d == {"v55"} and u == {"v44", "v38", "v11", "exec"}
    assert pair_sched.parse("s_mov_b32 s5, s[6:7]")[1] == {"s6", "s7"}
    for barrier in ("v_cmp_lt_u64_e32 vcc, v[42:43], v[6:7]", "v_cndmask_b32_e32 v7, v7, v43, vcc",
                    "s_nop 0", "s_cbranch_scc0 .LBB0_1", "v_readfirstlane_b32 s4, v1",
                    "v_add_u32_dpp v0, v1, v2 row_ror:4", "global_load_dword v1, v[2:3], off"):
        assert pair_sched.parse(barrier) is None, barrier


def test_deps_raw_war_waw():
    seg = ["v_add_u32_e64 v1, v2, v3",   # 0
           "v_xor_b32_e64 v4, v1, v5",   # 1 RAW v1 <- 0
           "v_add_u32_e64 v2, v6, v7",   # 2 WAR v2 -> after 0
           "v_add_u32_e64 v1, v8, v9"]   # 3 WAW v1 after 0, WAR after 1
    preds = pair_sched.deps([pair_sched.parse(s) for s in seg])
    assert preds == [set(), {0}, {0}, {0, 1}]


def _random_segment(rng, n=120, nreg=24):
    ops = ["v_alignbit_b32 v{d}, v{a}, v{a}, 7", "v_add3_u32 v{d}, v{a}, v{b}, v{c}",
           "v_bitop3_b32 v{d}, v{a}, v{b}, v{c} bitop3:0x96", "v_add_u32_e64 v{d}, v{a}, v{b}",
           "s_lshr_b32 s{d}, s{a}, 3", "v_add_u32_e64 v{d}, s{a}, v{b}"]
    out = []
    for _ in range(n):
        t = rng.choice(ops)
        out.append(t.format(d=rng.randrange(nreg), a=rng.randrange(nreg), b=rng.randrange(nreg),
                            c=rng.randrange(nreg)))
    return out


def _interpret(seg, order):
    """run the segment in `order` on symbolic registers: the final state
    must not depend on the order (every def sees the same inputs)."""
    state = {}
    for i in order:
        d, u = pair_sched.parse(seg[i])
        op = seg[i].split()[0]
        val = (op, tuple(sorted((r, state.get(r, r)) for r in u if r not in ("exec", "scc"))))
        for r in d:
            if r != "scc":
                state[r] = val
    return state


# (run, amax, bmax): the uncapped modes and the run caps the build ships
# (Makefile ISAPOST: --pair-sched=0 --sched-amax=5 --sched-bmax=4) and its
# A/B neighbours
SCHED_MODES = [(0, 0, 0), (2, 0, 0), (3, 0, 0), (0, 5, 4), (0, 5, 0), (0, 0, 4), (0, 3, 2), (0, 1, 1), (0, 8, 8)]


@pytest.mark.parametrize("run,amax,bmax", SCHED_MODES)
def test_schedule_keeps_semantics_on_random_segments(run, amax, bmax):
    rng = random.Random(440 + 17 * amax + bmax)
    for _ in range(30):
        seg = _random_segment(rng)
        order = pair_sched.schedule(seg, isa_post.issue_class, run, amax, bmax)
        assert sorted(order) == list(range(len(seg)))
        assert _interpret(seg, order) == _interpret(seg, range(len(seg)))


def _transitions(seq):
    v = [c for c in seq if c != "S"]
    return sum(1 for x, y in zip(v, v[1:]) if x == "A" and y == "B")


@pytest.mark.parametrize("amax,bmax", [(0, 0), (5, 4), (5, 0), (0, 4)])
def test_sticky_schedule_cuts_half_to_full_rate_transitions(amax, bmax):
    rng = random.Random(441)
    before = after = 0
    for _ in range(20):
        seg = _random_segment(rng, n=200, nreg=40)
        cls = [isa_post.issue_class(s) for s in seg]
        order = pair_sched.schedule(seg, isa_post.issue_class, 0, amax, bmax)
        before += _transitions(cls)
        after += _transitions([cls[i] for i in order])
    assert after < before * 0.8, (before, after)


def test_capped_runs_respect_their_caps_when_the_other_class_is_ready():
    """amax / bmax: a run of one class is cut at the cap whenever an op of
    the other class is ready -- on independent ops (always ready) the runs
    are exactly the caps (a segment opens with the full-rate class)."""
    seg = [f"v_alignbit_b32 v{i}, v{i}, v{i}, 7" for i in range(20)] + \
          [f"v_add_u32_e64 v{100 + i}, v{100 + i}, v{100 + i}" for i in range(20)]
    order = pair_sched.schedule(seg, isa_post.issue_class, 0, 5, 4)
    cls = "".join(isa_post.issue_class(seg[i]) for i in order)
    runs = [len(m.group(0)) for m in re.finditer(r"A+|B+", cls)]
    assert max(len(r) for r in re.findall(r"A+", cls)) <= 5 and max(len(r) for r in re.findall(r"B+", cls)) <= 4
    assert cls[0] == "B" and runs[:6] == [4, 5, 4, 5, 4, 5], cls  # full-rate first, then alternate at the caps


def _region(body):
    return [".LBB0_1:"] + ["\t" + s for s in body] + ["\ts_cbranch_scc0 .LBB0_1"]


def test_hazard_check_trips_on_a_shortened_dpp_distance():
    """the reorder may not move a VGPR write closer
    than HAZARD_WINDOW wait states to a DPP read right after the segment.
    Original order: v1 written first, then five independent ops; a schedule
    that emits the half-rate write last brings it next to the DPP op."""
    seg = ["v_alignbit_b32 v1, v1, v1, 7"] + [f"v_add_u32_e64 v{10 + i}, v{20 + i}, v{30 + i}" for i in range(5)]
    dpp = "v_add_u32_dpp v2, v1, v3 row_ror:4 row_mask:0xf bank_mask:0xf"
    order = [1, 2, 3, 4, 5, 0]
    with pytest.raises(pair_sched.HazardError, match="v1"):
        pair_sched.check_hazards(seg, order, [dpp], [])
    pair_sched.check_hazards(seg, list(range(6)), [dpp], [])       # original order: fine
    pair_sched.check_hazards(seg, order, ["v_cmp_lt_u32_e32 vcc, v1, v2"], [])  # plain VALU consumer: no wait
    # far enough away: the write still sits 6 wait states before the DPP op
    pair_sched.check_hazards(seg, order, ["s_nop 5", dpp], [])
    with pytest.raises(pair_sched.HazardError):
        pair_sched.check_hazards(seg, order, ["s_nop 3", dpp], [])
    # a VMEM read of the moved write and a readlane of it are checked alike
    for consumer in ("global_store_dword v[4:5], v1, off", "v_readlane_b32 s4, v1, 3"):
        with pytest.raises(pair_sched.HazardError):
            pair_sched.check_hazards(seg, order, [consumer], [])


def test_hazard_check_trips_on_a_read_moved_next_to_a_transcendental():
    seg = [f"v_add_u32_e64 v{10 + i}, v{20 + i}, v{30 + i}" for i in range(5)] + ["v_xor_b32_e64 v9, v1, v2"]
    order = [5, 0, 1, 2, 3, 4]
    with pytest.raises(pair_sched.HazardError, match="v1"):
        pair_sched.check_hazards(seg, order, [], ["v_exp_f32_e32 v1, v7"])
    pair_sched.check_hazards(seg, order, [], ["v_add_u32_e64 v1, v7, v8"])  # plain producer


def test_pass_never_emits_a_hazardous_reorder():
    """Through the pass itself: a segment whose schedule moves a half-rate
    write to its end, right before a DPP read of it, fails the build under
    --strict-hazards and otherwise keeps LLVM's order."""
    body = ["v_alignbit_b32 v1, v1, v1, 7"] + [f"v_add_u32_e64 v{10 + i}, v{20 + i}, v{30 + i}" for i in range(5)] + \
           ["v_add_u32_e64 v40, v41, v42", "v_add_u32_dpp v2, v1, v3 row_ror:4 row_mask:0xf bank_mask:0xf"]
    lines = _region(body)
    stats = {"sched_segments": 0, "sched_moved": 0}
    order = pair_sched.schedule(body[:7], isa_post.issue_class, 0, 0, 0)
    assert order.index(0) == 6  # the full-rate run goes first: the write lands next to the DPP read
    with pytest.raises(pair_sched.HazardError):
        pair_sched.pass_pair_sched(lines, [(0, len(lines) - 1)], isa_post.is_instr, isa_post.issue_class, stats, 0,
                                   strict=True)
    # the default keeps LLVM's order for that segment instead
    kept = pair_sched.pass_pair_sched(lines, [(0, len(lines) - 1)], isa_post.is_instr, isa_post.issue_class, stats, 0)
    assert kept == lines and stats["hazard_kept"] == 1
    # the same segment with the DPP read further away (a barrier and 5 wait states between) passes
    far = _region(body[:7] + ["v_cmp_lt_u32_e32 vcc, v1, v2", "s_nop 4", body[7]])
    pair_sched.pass_pair_sched(far, [(0, len(far) - 1)], isa_post.is_instr, isa_post.issue_class, stats, 0)
    assert stats["sched_segments"] >= 1


def test_shipped_post_pass_output_passes_the_hazard_check():
    """The shipped post-pass (Makefile ISAPOST) run on the build's compiler
    output reproduces build/p1hip_kernels.post.s byte for byte with the
    check in force (a segment the check rejects keeps LLVM's order)."""
    src = os.path.join(ROOT, "build", "p1hip_kernels.s")
    post = os.path.join(ROOT, "build", "p1hip_kernels.post.s")
    if not (os.path.exists(src) and os.path.exists(post)):
        pytest.skip("build/p1hip_kernels.s not built")
    mk = open(os.path.join(ROOT, "Makefile")).read()
    opts = next(ln for ln in mk.split("\n") if ln.startswith("ISAPOST ?=")).split("=", 1)[1].split()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "post.s")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_post.py"), src, out] + opts,
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-2000:]
        stats = json.loads(r.stderr.strip().split("\n")[-1])
        assert stats["hazard_checked"] >= stats["sched_segments"] > 0, stats
        assert open(out).read() == open(post).read()


def test_segments_stop_at_barriers():
    lines = ["\t.p2align 3", ".LBB0_1:", "\tv_add_u32_e64 v1, v2, v3", "\tv_alignbit_b32 v4, v4, v4, 7",
             "\tv_bitop3_b32 v5, v6, v7, v8 bitop3:0x96", "\tv_cmp_lt_u32_e32 vcc, v1, v5",
             "\tv_alignbit_b32 v9, v9, v9, 3", "\tv_add_u32_e64 v10, v11, v12", "\tv_alignbit_b32 v13, v13, v13, 5",
             "\ts_cbranch_scc0 .LBB0_1"]
    stats = {"sched_segments": 0, "sched_moved": 0}
    out = pair_sched.pass_pair_sched(lines, [(1, 9)], isa_post.is_instr, isa_post.issue_class, stats, 0)
    assert out[5] == lines[5] and out[9] == lines[9]           # barriers stay put
    assert sorted(out[2:5]) == sorted(lines[2:5])               # nothing crosses the compare
    assert sorted(out[6:9]) == sorted(lines[6:9])


def test_loop_regions_take_unconditional_back_edges():
    """A loop whose exit test comes before an unconditional back branch (the
    layout LLVM chose for the work-queue k_scan's MODE 7 block-0 loop) is a
    region too, so the post-pass schedules it and sets its priorities; the
    region ends at the last branch back to the header."""
    lines = [".LBB0_7:                               ; =>This Loop Header: Depth=1",
             "\tv_alignbit_b32 v1, v1, v1, 7", "\ts_cmp_eq_u32 s3, 10", "\ts_cbranch_scc1 .LBB0_9",
             "\tv_add_u32_e32 v2, v2, v3", "\ts_cbranch_scc0 .LBB0_7", "\tv_add_u32_e32 v4, v4, v3",
             "\ts_branch .LBB0_7", ".LBB0_9:", "\ts_endpgm"]
    assert isa_post.loop_regions(lines) == [(0, 7)]


def test_hoist_consts_moves_only_provably_invariant_moves():
    """isa_post --hoist-consts (builds without MachineLICM): a constant move
    leaves an innermost single-block loop only when it is the loop's one
    write of its register, nothing before it in the body names that
    register, and the header is entered only by its own back edge."""
    lines = ["\ts_mov_b32 s9, 0", ".LBB0_4:                               ; =>This Inner Loop Header: Depth=1",
             "\ts_mov_b32 s20, 0x428a2f98",       # hoistable
             "\tv_add_u32_e32 v1, s20, v1",
             "\ts_mov_b32 s21, 0x71374491",       # written twice: stays
             "\tv_add_u32_e32 v2, s21, v2",
             "\ts_mov_b32 s21, 0xb5c0fbcf",
             "\tv_add_u32_e32 v3, s22, v3",       # s22 read before its move: stays
             "\ts_mov_b32 s22, 0xe9b5dba5",
             "\ts_add_i32 s9, s9, 1",
             "\ts_cmp_lg_u32 s9, 10",
             "\ts_cbranch_scc1 .LBB0_4",
             "\ts_endpgm"]
    stats = {}
    out = isa_post.pass_hoist_consts(lines, stats)
    assert stats["consts_hoisted"] == 1
    assert out.index("\ts_mov_b32 s20, 0x428a2f98") < out.index(lines[1])
    assert "\ts_mov_b32 s21, 0x71374491" in out[out.index(lines[1]):]
    assert "\ts_mov_b32 s22, 0xe9b5dba5" in out[out.index(lines[1]):]
    # a branch into the header from outside the loop: nothing moves
    entered = lines[:1] + ["\ts_cbranch_scc0 .LBB0_4"] + lines[1:]
    stats = {}
    assert isa_post.pass_hoist_consts(entered, stats) == entered and not stats.get("consts_hoisted")
