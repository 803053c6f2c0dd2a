"""Dump the per-nonce (innermost, largest) loop of one fast variant of
k_scan, built through the shipped pipeline (tools/variant_report.py
build steps), one line per instruction: "addr size class text" with
class A = half-rate VALU, B = full-rate VALU, S = scalar.  Input of
tools/gen_loopbench.py.  Test tool, not product.

usage: loop_dump.py FV MODE TRAIL OUT [--isapost "..."]"""
import argparse
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import variant_report as vr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fv", type=int)
    ap.add_argument("mode", type=int)
    ap.add_argument("trail", choices=["true", "false"])
    ap.add_argument("out")
    ap.add_argument("--isapost", default="--no-e64 --align-loops=3 --loop-offset=4 --pair-sched=0 --sched-amax=5 --sched-bmax=4 --prio=0,1")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        inc = os.path.join(td, "v.inc")
        open(inc, "w").write(f"P1_CASE({a.fv}, {a.mode}, {a.trail})\n")
        s = os.path.join(td, "k.s")
        subprocess.run([vr.HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-o", s,
                        f"-DP1_VARIANTS_INC=\"{inc}\"", os.path.join(vr.ROOT, "p1_amd/csrc/p1hip_kernels.hip")],
                       check=True, capture_output=True)
        post = os.path.join(td, "k.post.s")
        subprocess.run([sys.executable, os.path.join(vr.ROOT, "tools/isa_post.py"), s, post] + a.isapost.split(),
                       check=True, capture_output=True)
        o, co = os.path.join(td, "k.o"), os.path.join(td, "k.co")
        subprocess.run([f"{vr.LLVM}/clang", "-cc1as", "-triple", "amdgcn-amd-amdhsa", "-filetype", "obj",
                        "-target-cpu", "gfx950", "-mrelocation-model", "pic", "-o", o, post], check=True)
        subprocess.run([f"{vr.LLVM}/ld.lld", "-m", "elf64_amdgpu", "--no-undefined", "-shared", "-o", co, o],
                       check=True)
        ins, inner, _ = vr.loops_of(co)
    big = max(inner, key=lambda l: l[1] - l[0])
    with open(a.out, "w") as f:
        for addr, sz, t in ins:
            if big[0] <= addr <= big[1]:
                op = t.split()[0]
                cls = "A" if op in vr.HALF_RATE else ("B" if op.startswith("v_") else "S")
                f.write(f"{addr:x} {sz} {cls} {t}\n")


if __name__ == "__main__":
    main()
