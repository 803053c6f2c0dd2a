"""tools/pair_sched.py: the post-RA reordering of loop segments for dual
issue keeps every register dependency and never moves an instruction across
a barrier.  CPU only."""
import os
import random
import sys

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


def test_schedule_keeps_semantics_on_random_segments():
    rng = random.Random(440)
    for mode in (0, 2, 3):
        for _ in range(30):
            seg = _random_segment(rng)
            order = pair_sched.schedule(seg, isa_post.issue_class, mode)
            assert sorted(order) == list(range(len(seg)))
            assert _interpret(seg, order) == _interpret(seg, range(len(seg)))


def test_sticky_schedule_cuts_half_to_full_rate_transitions():
    rng = random.Random(441)
    before = after = 0
    for _ in range(20):
        seg = _random_segment(rng, n=200, nreg=40)
        cls = [isa_post.issue_class(s) for s in seg]
        order = pair_sched.schedule(seg, isa_post.issue_class, 0)

        def transitions(seq):
            v = [c for c in seq if c != "S"]
            return sum(1 for x, y in zip(v, v[1:]) if x == "A" and y == "B")
        before += transitions(cls)
        after += transitions([cls[i] for i in order])
    assert after < before * 0.8, (before, after)


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
