#!/usr/bin/env python3
"""Report the byte parity of 8-byte instructions inside the loops of a gfx950
code object (evidence for tools/isa_post.py --loop-parity).

usage: check_parity.py CODE_OBJECT [kernel]
A loop = the address range [target, branch] of every backward s_cbranch.
Prints JSON: loops, 8-byte instructions in loops, how many sit at 4 mod 8."""
import json
import re
import subprocess
import sys

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def main():
    co = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else "k_scan"
    dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", co], capture_output=True, text=True).stdout.split("\n")
    ins = []  # (addr, size, text)
    on = False
    base = 0
    for ln in dis:
        mh = re.match(r"^([0-9a-f]+) <(.*)>:", ln)
        if mh:
            on = mh.group(2) == kern
            base = int(mh.group(1), 16)
            continue
        m = re.search(r"^\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):\s*((?:[0-9A-Fa-f]{8}\s*)+)(<.*>)?$", ln)
        if on and m:
            ins.append((int(m.group(2), 16), 4 * len(m.group(3).split()), m.group(1)))
    del base
    loops = []
    for a, sz, t in ins:
        m = re.match(r"s_cbranch_\w+\s+(\d+)", t)
        if m:
            off = int(m.group(1))
            off = off - 65536 if off >= 32768 else off  # simm16, dwords from the next instruction
            tgt = a + 4 + 4 * off
            if tgt < a:
                loops.append((tgt, a))
    n8 = good = 0
    per = []
    for lo, hi in loops:
        k8 = [(a, sz) for a, sz, t in ins if lo <= a <= hi and sz == 8]
        g = sum(1 for a, sz in k8 if a % 8 == 4)
        n8 += len(k8)
        good += g
        per.append({"start": hex(lo), "bytes": hi - lo + 4, "n8": len(k8), "at_4_mod_8": g})
    print(json.dumps({"kernel": kern, "loops": len(loops), "n8_in_loops": n8, "at_4_mod_8": good,
                      "frac": good / n8 if n8 else None,
                      "worst": sorted(per, key=lambda p: p["at_4_mod_8"] / max(1, p["n8"]))[:3]}))


if __name__ == "__main__":
    main()
