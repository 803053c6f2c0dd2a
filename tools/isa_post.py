#!/usr/bin/env python3
"""Peephole pass over the gfx950 assembly of the scan kernels.

usage: isa_post.py IN.s OUT.s [--no-e64] [--drop-asm-nops]

1. VOP2 -> VOP3 encoding of full-rate integer ops (v_add_u32_e32 ->
   v_add_u32_e64, likewise lshrrev/lshlrev/xor/and/or/sub).  Same operation,
   same result; measured on MI355X (tools/valu_runs, profiles/r01m_valu_runs.jsonl):
   in a stream mixed with half-rate VOP3 ops (v_alignbit_b32, v_add3_u32) a
   VOP2-encoded add/xor/shift costs ~4.1 SIMD cycles per wave instruction, the
   VOP3-encoded one ~3.1 (and bitop3 ~3.1).  LLVM always shrinks to VOP2 when
   it can and has no switch to keep the long form.  Only register / inline-
   constant operands are converted (gfx950 VOP3 takes no literal).
2. --drop-asm-nops: remove the `s_nop 0` LLVM's hazard recognizer puts after
   an inline-asm block whose next instruction reads the block's result.  It
   must assume the asm may be a transcendental op (1 wait state before a
   dependent VALU on gfx940+); our blocks are single v_bitop3_b32, which LLVM
   itself schedules back-to-back with its consumers when it emits the same
   instruction (no wait state).

Prints a one-line JSON summary of what changed to stderr.
"""
import json
import re
import sys

E32_OPS = ("v_add_u32", "v_sub_u32", "v_subrev_u32", "v_lshrrev_b32", "v_lshlrev_b32", "v_xor_b32", "v_and_b32",
           "v_or_b32")
RE_E32 = re.compile(r"^(\s*)(" + "|".join(E32_OPS) + r")_e32(\s+)(.*)$")
# plain VALU consumers (no DPP/SDWA/readlane/memory): no wait state after a VALU write
SAFE_NEXT = re.compile(r"^(v_add3_u32|v_add_u32_e(32|64)|v_alignbit_b32|v_lshrrev_b32_e(32|64)|v_xor_b32_e(32|64)|"
                       r"v_bitop3_b32|v_cndmask_b32_e(32|64))\s(?!.*(dpp|sdwa|row_|quad_))")
REG = re.compile(r"^(v\d+|s\d+|vcc_lo|vcc_hi|exec_lo|exec_hi|m0)$")


def inline_const(tok):
    try:
        v = int(tok, 0)
    except ValueError:
        return False
    return -16 <= v <= 64


def convertible(ops):
    parts = [p.strip() for p in ops.split(",")]
    if len(parts) != 3:
        return False
    return all(REG.match(p) or inline_const(p) for p in parts)


def main():
    src, dst = sys.argv[1], sys.argv[2]
    e64 = "--no-e64" not in sys.argv
    drop_nops = "--drop-asm-nops" in sys.argv
    align = 0
    offset = 0
    for a in sys.argv:
        if a.startswith("--align-loops="):
            align = int(a.split("=")[1])
        if a.startswith("--loop-offset="):
            offset = int(a.split("=")[1])
    lines = open(src).read().split("\n")
    out = []
    n_e64 = n_nop = 0
    last_asm_bitop3 = False  # previous real instruction came from a v_bitop3 inline-asm block
    in_asm = False

    def next_real(i):
        for ln2 in lines[i + 1:]:
            t = ln2.strip()
            if not t or t.startswith(";"):
                continue
            return t
        return ""

    def is_loop_header(i):
        # the label line and the comment-only lines that follow it
        if "Inner Loop Header" in lines[i]:
            return True
        for ln2 in lines[i + 1:]:
            t = ln2.strip()
            if t and not t.startswith(";"):
                return False
            if "Inner Loop Header" in t:
                return True
        return False

    n_align = 0
    for i, ln in enumerate(lines):
        s = ln.strip()
        if align and re.match(r"^\.LBB\d+_\d+:", ln) and is_loop_header(i):
            out.append(f"\t.p2align {align}")
            out += ["\ts_nop 0"] * (offset // 4)
            n_align += 1
        if s == ";;#ASMSTART":
            in_asm = True
            out.append(ln)
            continue
        if s == ";;#ASMEND":
            in_asm = False
            out.append(ln)
            continue
        if not s or s.startswith(";"):
            out.append(ln)
            continue
        if in_asm:
            last_asm_bitop3 = s.startswith("v_bitop3_b32")
            out.append(ln)
            continue
        if drop_nops and last_asm_bitop3 and s == "s_nop 0" and SAFE_NEXT.match(next_real(i)):
            n_nop += 1
            continue
        last_asm_bitop3 = False
        m = RE_E32.match(ln)
        if e64 and m and convertible(m.group(4).split(";")[0]):
            ln = f"{m.group(1)}{m.group(2)}_e64{m.group(3)}{m.group(4)}"
            n_e64 += 1
        out.append(ln)
    open(dst, "w").write("\n".join(out))
    print(json.dumps({"e64_converted": n_e64, "asm_nops_dropped": n_nop, "loops_aligned": n_align}), file=sys.stderr)


if __name__ == "__main__":
    main()
