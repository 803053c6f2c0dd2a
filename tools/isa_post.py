#!/usr/bin/env python3
"""Peephole pass over the gfx950 assembly of the scan kernels (build step,
Makefile: build/p1hip_kernels.s -> build/p1hip_kernels.post.s).

usage: isa_post.py IN.s OUT.s [--no-e64] [--drop-asm-nops]
                               [--align-loops=P --loop-offset=B] [--loop-parity]
                               [--hoist-consts] [--pair-sched=0 [--sched-amax=K] [--sched-bmax=K] [--strict-hazards]]
                               [--prio=PB,PA]
                               A/B only: [--ab-nop=N [--nop-where=ab|abb|ba] [--ab-nop-table=..]]
                                         [--ba-nop=N] [--split-add3=F]
shipped: the Makefile's ISAPOST line is the one source of the shipped
  options (round 6: --no-e64 --align-loops=3 --loop-offset=4
  --pair-sched=0 --sched-amax=5 --sched-bmax=4 --strict-hazards --prio=0,1;
  no --loop-parity).
  Items 1, 2, 4 and 5 below are A/B options kept for the record: the VOP3
  widening (1) and the parity rule (2) were retired in round 5 (DESIGN.md 4
  "The parity rule is retired"); the scheduler (3) also checks that no
  reorder shortens a wait-state distance LLVM relied on (tools/pair_sched.py
  check_hazards: with --strict-hazards, shipped, the build fails if one
  does; without it that segment keeps LLVM's order).

What it does and why (measurements: tools/valu_runs on MI355X,
profiles/r01s_valu_runs.jsonl, profiles/r01v_valu_runs.jsonl, and the
scan-kernel A/Bs in profiles/r01n_e64_ab.jsonl, profiles/r01r_loop_offset_sweep.jsonl):

1. (A/B, retired: --no-e64 ships) VOP2 -> VOP3 encoding of full-rate integer ops (v_add_u32_e32 ->
   v_add_u32_e64, likewise lshrrev/lshlrev/xor/and/or/sub).  Same operation,
   same result.  LLVM always shrinks to the 4-byte VOP2 form; in a stream
   mixed with half-rate VOP3 ops (v_alignbit_b32, v_add3_u32) every 4-byte
   instruction shifts the byte parity of the 8-byte ones that follow (2).
   Only register / inline-constant operands are converted (gfx950 VOP3 takes
   no literal).
2. (the --loop-parity part is an A/B option, retired) Byte parity of 8-byte
   instructions in hot loops.  A wave stream that mixes
   half-rate VOP3 (4.3 SIMD cycles per wave instruction alone) with full-rate
   VOP3 (2.7) issues at the additive rate only when the 8-byte instructions
   sit at addresses = 4 (mod 8); at 0 (mod 8) EVERY instruction of the mix
   costs ~4.2 cycles (the full-rate ones lose their advantage).  Measured on
   the c2 scan kernel: loop start at 4 mod 8 -> 36.3 GH/s, at 0 mod 8 ->
   32.1 GH/s, every 4-byte step of a 64-byte sweep.
   --align-loops=3 --loop-offset=4 puts each loop label at 4 (mod 8)
   (`.p2align 3` + one `s_nop 0` executed once on loop entry).
   --loop-parity additionally walks each loop body with exact
   instruction sizes (from llvm-mc) and restores the parity after every
   4-byte instruction that breaks it: by widening the preceding 4-byte VALU
   (VOP1/VOP2/VOPC e32 -> e64, same operands) where possible, else by
   inserting one `s_nop 0` before the next 8-byte instruction.
3. --pair-sched=0 (tools/pair_sched.py) reorders every straight-line
   segment of a loop body into runs of one issue class within its register
   dependency DAG (half-rate runs capped at --sched-amax, full-rate runs at
   --sched-bmax ops when the other class is ready), and --prio=PB,PA puts
   `s_setprio PA` before each half-rate run and `s_setprio PB` before each
   full-rate run: gfx950 issues a half-rate op beside a full-rate op of a
   LOWER-priority wave in one 4-cycle slot, never beside another half-rate
   op (DESIGN.md 4 "Dual issue"; c4 0.649 -> 0.928 of the int32 peak).
   --split-add3=F (A/B) splits F x the half-rate/full-rate imbalance of
   VGPR-only v_add3_u32 into two full-rate adds.
4. --ab-nop[=N] (A/B; superseded by --prio): one `s_nop N` before every full-rate VALU op
   that directly follows a half-rate one in a loop body (no scalar
   instruction between them).  gfx950 issues two full-rate VALU ops of two
   different waves in one 4-cycle slot (SQ_ACTIVE_INST_VALU2) but a
   half-rate op alone; with the oldest wave issuing every slot, the waves
   behind it rarely hold a full-rate op when it does, and a scalar filler
   after the half-rate op hands the slot to them (tools/gen_dual.py:
   A,nop,B pairs 93% of its B ops where A,B pairs 0-56%).  A/B option.
5. --drop-asm-nops: remove the `s_nop 0` LLVM's hazard recognizer puts after
   an inline-asm block whose next instruction reads the block's result.  For
   inline asm it must assume a dst_sel (16-bit) forwarding hazard on gfx950;
   our blocks are single 32-bit v_bitop3_b32, which LLVM itself issues
   back-to-back with its consumers when it selects the instruction.  Off by
   default: it changes code addresses (see 2) and is not needed for speed.

Prints a one-line JSON summary of what changed to stderr.
"""
import json
import os
sys_path_here = os.path.dirname(os.path.abspath(__file__))
import re
import subprocess
import sys
import tempfile

E32_OPS = ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_lshrrev_b32", "v_lshlrev_b32", "v_xor_b32", "v_and_b32",
           "v_or_b32")
RE_E32 = re.compile(r"^(\s*)(" + "|".join(E32_OPS) + r")_e32(\s+)(.*)$")
# any VOP1/VOP2/VOPC in its 4-byte form (parity pass may widen it)
RE_ANY_E32 = re.compile(r"^(\s*)(v_[a-z0-9_]+)_e32(\s+)(.*)$")
# plain VALU consumers (no DPP/SDWA/readlane/memory): no wait state after a VALU write
SAFE_NEXT = re.compile(r"^(v_add3_u32|v_add_u32_e(32|64)|v_alignbit_b32|v_lshrrev_b32_e(32|64)|v_xor_b32_e(32|64)|"
                       r"v_bitop3_b32|v_cndmask_b32_e(32|64))\s(?!.*(dpp|sdwa|row_|quad_))")
REG = re.compile(r"^(v\d+|s\d+|vcc_lo|vcc_hi|vcc|exec_lo|exec_hi|m0|v\[\d+:\d+\]|s\[\d+:\d+\])$")
RE_LABEL = re.compile(r"^(\.LBB\d+_\d+):")
RE_BRANCH = re.compile(r"^s_cbranch_\w+\s+(\.LBB\d+_\d+)")
# a loop's back edge: conditional, or an unconditional s_branch when LLVM
# puts the exit test before the latch (the round-6 work-queue k_scan lays
# out MODE 7's and the split modes' outer loops that way)
RE_BACK = re.compile(r"^s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)")
LLVM_MC = os.environ.get("LLVM_MC", "/opt/rocm/lib/llvm/bin/llvm-mc")


def inline_const(tok):
    try:
        v = int(tok, 0)
    except ValueError:
        return False
    return -16 <= v <= 64


def operands(text):
    return [p.strip() for p in text.split(";")[0].split(",")]


def convertible(ops):
    parts = operands(ops)
    if len(parts) != 3:
        return False
    return all(REG.match(p) or inline_const(p) for p in parts)


def widen(line):
    """4-byte VOP1/VOP2/VOPC line -> the same instruction in its 8-byte VOP3
    form, or None when that form cannot hold the operands."""
    m = RE_ANY_E32.match(line)
    if not m or "dpp" in line or "sdwa" in line:
        return None
    parts = operands(m.group(4))
    if not all(REG.match(p) or inline_const(p) for p in parts):
        return None
    return f"{m.group(1)}{m.group(2)}_e64{m.group(3)}{m.group(4)}"


def is_instr(s):
    return bool(s) and not s.startswith((";", ".")) and not RE_LABEL.match(s)


def sizes_of(instrs, cpu="gfx950"):
    """Encoded size in bytes of each instruction line (one llvm-mc run)."""
    if not instrs:
        return []
    with tempfile.NamedTemporaryFile("w", suffix=".s", delete=False) as f:
        f.write("\n".join(instrs) + "\n")
        path = f.name
    try:
        r = subprocess.run([LLVM_MC, "-arch=amdgcn", f"-mcpu={cpu}", "-show-encoding", path],
                           capture_output=True, text=True)
    finally:
        os.unlink(path)
    enc = [ln for ln in r.stdout.split("\n") if "; encoding: [" in ln]
    if len(enc) != len(instrs):
        raise SystemExit(f"isa_post: llvm-mc sized {len(enc)} of {len(instrs)} instructions:\n{r.stderr[-2000:]}")
    return [len(e.split("; encoding: [")[1].rstrip("]").split(",")) for e in enc]


def loop_headers(lines, tag="Loop Header"):
    """Indices of loop header labels (LLVM's loop comments): every loop with
    the default tag, innermost loops only with tag="Inner Loop Header"."""
    hdr = []
    for i, ln in enumerate(lines):
        if not RE_LABEL.match(ln):
            continue
        if tag in ln:
            hdr.append(i)
            continue
        for ln2 in lines[i + 1:]:
            t = ln2.strip()
            if t and not t.startswith(";"):
                break
            if tag in t:
                hdr.append(i)
                break
    return hdr


def pass_encode(lines, e64, drop_nops, stats):
    out = []
    last_asm_bitop3 = False
    in_asm = False

    def next_real(i):
        for ln2 in lines[i + 1:]:
            t = ln2.strip()
            if not t or t.startswith(";"):
                continue
            return t
        return ""

    for i, ln in enumerate(lines):
        s = ln.strip()
        if s == ";;#ASMSTART":
            in_asm = True
        elif s == ";;#ASMEND":
            in_asm = False
        elif s and not s.startswith(";"):
            if in_asm:
                last_asm_bitop3 = s.startswith("v_bitop3_b32")
            elif drop_nops and last_asm_bitop3 and s == "s_nop 0" and SAFE_NEXT.match(next_real(i)):
                stats["asm_nops_dropped"] += 1
                continue
            else:
                last_asm_bitop3 = False
                m = RE_E32.match(ln)
                if e64 and m and convertible(m.group(4)):
                    ln = f"{m.group(1)}{m.group(2)}_e64{m.group(3)}{m.group(4)}"
                    stats["e64_converted"] += 1
        out.append(ln)
    return out


def pass_align(lines, align, offset, stats):
    hdr = set(loop_headers(lines))
    out = []
    for i, ln in enumerate(lines):
        if i in hdr:
            out.append(f"\t.p2align {align}")
            out += ["\ts_nop 0"] * (offset // 4)
            stats["loops_aligned"] += 1
        out.append(ln)
    return out


HALF_RATE = {"v_alignbit_b32", "v_add3_u32", "v_alignbyte_b32", "v_perm_b32", "v_xad_u32", "v_or3_b32",
             "v_lshl_or_b32", "v_lshl_add_u32", "v_add_lshl_u32", "v_and_or_b32", "v_bfi_b32", "v_bfe_u32",
             "v_mad_u32_u24", "v_pk_add_u16", "v_cndmask_b32_e64"}
RE_SGPR_OP = re.compile(r"(^|[\s,])s(\d+|\[\d+:\d+\])\b")


def issue_class(ins):
    """'A' half-rate VALU (3-input VOP3 integer ops; a VOP3 op with an SGPR
    source, tools/gen_dual.py kind k), 'B' full-rate VALU, 'S' anything else"""
    op, _, ops = ins.partition(" ")
    if not op.startswith("v_"):
        return "S"
    if op in HALF_RATE:
        return "A"
    srcs = ",".join(operands(ops)[1:])
    if (op.endswith("_e64") or op.startswith("v_bitop3")) and RE_SGPR_OP.search(srcs):
        return "A"
    return "B"


def loop_regions(lines):
    """(header line, back-edge line) of every loop laid out header first: the
    last branch to the header within 40,000 lines, conditional or not"""
    regions = []
    for h in loop_headers(lines):
        label = RE_LABEL.match(lines[h]).group(1)
        for j in range(min(len(lines), h + 40000) - 1, h, -1):
            m = RE_BACK.match(lines[j].strip())
            if m and m.group(1) == label:
                regions.append((h, j))
                break
    return regions


def pass_ab_nop(lines, nop, stats, where="ab", table=None):
    """where: 'ab' = before a full-rate op after a half-rate one; 'abb' = the
    same, only when the full-rate op starts a run of at least two; 'ba' =
    before a half-rate op after a full-rate one.  table (ab only): the wait
    by run lengths, {(A-run 1 or 2+, B-run 1 or 2+): N or -1 for none}."""
    inside = set()
    for a, b in loop_regions(lines):
        inside.update(range(a + 1, b + 1))
    cls = {i: issue_class(lines[i].strip()) for i in inside if is_instr(lines[i].strip())}

    def next_cls(i):
        for j in range(i + 1, len(lines)):
            if j in cls:
                return cls[j]
            if RE_LABEL.match(lines[j].strip()):
                return None
        return None

    out, last, arun = [], None, 0
    for i, ln in enumerate(lines):
        s = ln.strip()
        if i in cls:
            c = cls[i]
            hit = {"ab": c == "B" and last == "A",
                   "abb": c == "B" and last == "A" and next_cls(i) == "B",
                   "ba": c == "A" and last == "B"}[where]
            n = nop
            if hit and table is not None:
                n = table[(min(arun, 2), 2 if next_cls(i) == "B" else 1)]
                hit = n >= 0
            if hit:
                out.append(f"\ts_nop {n}")
                stats["ab_nops"] += 1
            arun = arun + 1 if (c == "A" and last == "A") else (1 if c == "A" else 0)
            last = c
        elif RE_LABEL.match(s):
            last, arun = None, 0
        out.append(ln)
    return out


RE_ADD3 = re.compile(r"^v_add3_u32\s+(v\d+),\s*(v\d+),\s*(v\d+),\s*(v\d+)\s*$")


def split_add3(ins):
    """v_add3_u32 d, a, b, c (VGPR operands) -> two full-rate v_add_u32_e64,
    the destination as the intermediate (read before it is overwritten)."""
    m = RE_ADD3.match(ins.split(";")[0].strip())
    if not m:
        return None
    d, a, b, c = m.groups()
    for x, y, z in ((a, b, c), (a, c, b), (b, c, a)):
        if d != z:
            return [f"v_add_u32_e64 {d}, {x}, {y}", f"v_add_u32_e64 {d}, {d}, {z}"]
    return None


def pass_split_add3(lines, frac, stats):
    """A/B option --split-add3=F: in each innermost loop, split F x (A - B)/3
    of its VGPR-only v_add3_u32 (evenly spread) into two full-rate adds, so
    that half-rate and full-rate ops balance (one of each per issue slot,
    DESIGN.md 4 "Dual issue")."""
    regions = loop_regions(lines)
    inner = [r for r in regions if not any(o != r and r[0] < o[0] and o[1] < r[1] for o in regions)]
    todo = set()
    for a, b in inner:
        idx = [k for k in range(a + 1, b + 1) if is_instr(lines[k].strip())]
        cls = [issue_class(lines[k].strip()) for k in idx]
        na, nb = cls.count("A"), cls.count("B")
        cand = [k for k in idx if split_add3(lines[k].strip())]
        budget = min(len(cand), max(0, int(round(frac * (na - nb) / 3.0))))
        if budget:
            step = len(cand) / budget
            todo.update(cand[int(i * step)] for i in range(budget))
    out = []
    for i, ln in enumerate(lines):
        if i in todo:
            out += ["\t" + x for x in split_add3(ln.strip())]
            stats["add3_split"] = stats.get("add3_split", 0) + 1
        else:
            out.append(ln)
    return out


RE_CONST_MOV = re.compile(r"^s_mov_b32\s+(s\d+),\s*(0x[0-9a-fA-F]+|-?\d+)\s*$")
NO_DEF_OPS = re.compile(r"^(s_cmp|s_cbranch|s_branch|s_waitcnt|s_nop|s_setprio|s_barrier|s_endpgm|s_sleep|"
                        r"global_store|buffer_store|flat_store|scratch_store|ds_write|s_store|s_dcache)")


def pass_hoist_consts(lines, stats):
    """A/B option --hoist-consts (for builds compiled without MachineLICM):
    move `s_mov_b32 sN, <imm>` out of every innermost loop to just before
    its header when that is provably the same program -- the loop is one
    basic block entered only by falling into its header (every branch to
    the header is the loop's own back edge), the move is the loop's only
    write of sN and nothing in the body names sN before it.  The body runs
    at least once, so sN holds the same constant after the loop too."""
    import pair_sched

    regions = loop_regions(lines)
    inner = [r for r in regions if not any(o != r and r[0] < o[0] and o[1] < r[1] for o in regions)]
    refs = {}
    for k, ln in enumerate(lines):
        m = re.search(r"\bs_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", ln)
        if m:
            refs.setdefault(m.group(1), []).append(k)
    move = {}  # line index -> header line index
    for a, b in inner:
        label = RE_LABEL.match(lines[a]).group(1)
        if any(not (a < k <= b) for k in refs.get(label, [])):
            continue
        body = [k for k in range(a + 1, b + 1) if lines[k].strip() and not lines[k].strip().startswith(";")]
        if any(RE_LABEL.match(lines[k].strip()) for k in body):
            continue
        seen = set()     # registers named so far in the body
        defs = {}        # register -> number of writes in the body
        for k in body:
            t = lines[k].strip().split(";")[0].strip()
            op, _, ops = t.partition(" ")
            first = ops.split(",")[0] if ops else ""
            if not NO_DEF_OPS.match(op):
                for r in pair_sched.regs(first):
                    defs[r] = defs.get(r, 0) + 1
        for k in body:
            t = lines[k].strip().split(";")[0].strip()
            m = RE_CONST_MOV.match(t)
            if m and m.group(1) not in seen and defs.get(m.group(1)) == 1:
                move[k] = a
            seen |= pair_sched.regs(t.partition(" ")[2])
    out = []
    hoist_at = {}
    for k, h in move.items():
        hoist_at.setdefault(h, []).append(lines[k])
    for i, ln in enumerate(lines):
        if i in move:
            continue
        if i in hoist_at:
            out += hoist_at[i]
            stats["consts_hoisted"] = stats.get("consts_hoisted", 0) + len(hoist_at[i])
        out.append(ln)
    return out


def pass_prio(lines, prio_b, prio_a, stats):
    """A/B option --prio=PB,PA: `s_setprio PB` before the first full-rate op
    of every run and `s_setprio PA` before the first half-rate op of every
    run inside the loop bodies (the issue arbiter prefers the higher
    priority, then the older wave)."""
    inside = set()
    for a, b in loop_regions(lines):
        inside.update(range(a + 1, b + 1))
    out, last = [], None
    for i, ln in enumerate(lines):
        s = ln.strip()
        if i in inside and is_instr(s):
            c = issue_class(s)
            if c in "AB" and c != last:
                out.append(f"\ts_setprio {prio_b if c == 'B' else prio_a}")
                stats["prio_switches"] = stats.get("prio_switches", 0) + 1
            if c in "AB":
                last = c
        elif RE_LABEL.match(s):
            last = None
        out.append(ln)
    return out


def pass_parity(lines, stats):
    """Loop bodies (label .. branch back to it) start at 4 mod 8 (pass_align
    with offset 4); keep every 8-byte instruction in them at 4 mod 8.  Loops
    nest: a line belongs to its innermost loop, whose header re-synchronises
    the position; an outer loop's own instructions (e.g. MODE 7's block-0
    update around its table loop) continue from where its inner loop ends."""
    regions = []
    for h in loop_headers(lines):
        label = RE_LABEL.match(lines[h]).group(1)
        for j in range(h + 1, min(len(lines), h + 40000)):
            m = RE_BRANCH.match(lines[j].strip())
            if m and m.group(1) == label:
                regions.append((h, j))
                break
    body_idx = [k for a, b in regions for k in range(a + 1, b + 1) if is_instr(lines[k].strip())]
    size = dict(zip(body_idx, sizes_of([lines[k].strip() for k in body_idx])))
    in_region = {}
    for a, b in sorted(regions, key=lambda r: r[0] - r[1]):  # outermost first: inner loops overwrite
        for k in range(a + 1, b + 1):
            in_region[k] = a
    out = []
    pos = None
    last_small = None  # index in `out` of the last 4-byte instruction since the last 8-byte one
    for i, ln in enumerate(lines):
        if i in in_region and i == in_region[i] + 1:
            pos, last_small = 4, None
        if i not in in_region or i not in size:
            out.append(ln)
            continue
        sz = size[i]
        if sz == 8 and pos % 8 == 0:
            w = widen(out[last_small]) if last_small is not None else None
            if w is not None:
                out[last_small] = w
                stats["parity_widened"] += 1
            else:
                out.append("\ts_nop 0")
                stats["parity_nops"] += 1
            pos += 4
        out.append(ln)
        pos += sz
        last_small = len(out) - 1 if sz == 4 and ln.strip().startswith("v_") else (
            last_small if sz == 4 else None)
    return out


def main():
    sys.path.insert(0, sys_path_here)
    src, dst = sys.argv[1], sys.argv[2]
    args = sys.argv[3:]
    opt = {a.split("=")[0]: (a.split("=")[1] if "=" in a else True) for a in args}
    stats = {"e64_converted": 0, "asm_nops_dropped": 0, "loops_aligned": 0, "parity_widened": 0, "parity_nops": 0,
             "ab_nops": 0}
    lines = open(src).read().split("\n")
    lines = pass_encode(lines, "--no-e64" not in opt, "--drop-asm-nops" in opt, stats)
    if "--hoist-consts" in opt:
        lines = pass_hoist_consts(lines, stats)
    if "--align-loops" in opt:
        lines = pass_align(lines, int(opt["--align-loops"]), int(opt.get("--loop-offset", 0)), stats)
    if "--split-add3" in opt:
        lines = pass_split_add3(lines, float(opt["--split-add3"]), stats)
    if "--pair-sched" in opt:
        import pair_sched
        stats.update(sched_segments=0, sched_moved=0)
        lines = pair_sched.pass_pair_sched(lines, loop_regions(lines), is_instr, issue_class, stats,
                                           3 if opt["--pair-sched"] is True else int(opt["--pair-sched"]),
                                           int(opt.get("--sched-amax", 0)), int(opt.get("--sched-bmax", 0)),
                                           strict="--strict-hazards" in opt)
    if "--ab-nop" in opt:
        table = None
        if "--ab-nop-table" in opt:  # N11,N12,N21,N22: (A-run 1|2+, B-run 1|2+)
            v = [int(x) for x in opt["--ab-nop-table"].split(",")]
            table = {(1, 1): v[0], (1, 2): v[1], (2, 1): v[2], (2, 2): v[3]}
        lines = pass_ab_nop(lines, 0 if opt["--ab-nop"] is True else int(opt["--ab-nop"]), stats,
                            opt.get("--nop-where", "ab"), table)
    if "--prio" in opt:
        pb, pa = (int(x) for x in opt["--prio"].split(","))
        lines = pass_prio(lines, pb, pa, stats)
    if "--ba-nop" in opt:
        lines = pass_ab_nop(lines, 0 if opt["--ba-nop"] is True else int(opt["--ba-nop"]), stats, "ba")
    if "--loop-parity" in opt:
        if opt.get("--align-loops") != "3" or opt.get("--loop-offset") != "4":
            raise SystemExit("--loop-parity needs --align-loops=3 --loop-offset=4")
        lines = pass_parity(lines, stats)
    open(dst, "w").write("\n".join(lines))
    print(json.dumps(stats), file=sys.stderr)


if __name__ == "__main__":
    main()
