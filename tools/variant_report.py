#!/usr/bin/env python3
"""Per-variant report of the fast scan kernel: for every (FV, NV, TRAIL) of
p1_amd/csrc/fast_variants.inc, build k_scan with only that variant through
the shipped pipeline (hipcc -S -> tools/isa_post.py -> code object) and read

  * .vgpr_count / .sgpr_count / .sgpr_spill_count and the waves per SIMD
    they admit (VGPR: 512 / vgprs; SGPR: MI355X_MICROARCH.md:225-226,
    blocks of 256 threads per CU = floor(800 / (ceil(sgpr/16)*16 + 16)));
  * the innermost per-nonce loop (largest loop containing no other loop):
    VALU instructions by issue class -- half-rate "A" (v_alignbit_b32,
    v_add3_u32 and the other 3-input VOP3 integer ops) and full-rate "B" --
    SALU instructions, bytes, and how many 8-byte instructions sit at
    4 (mod 8);
  * the enclosing loop's own instructions (inner loop excluded), per trip;
  * a predicted rate from the measured issue costs (A 4.37,
    B 2.66 SIMD cycles per wave instruction at 4 waves/SIMD) at 2.35 GHz.

usage: variant_report.py [--jobs N] [--only FV,NV,TR ...] [--waves W] > out.jsonl
       variant_report.py --explain [report.jsonl ...]   (FV-floor decomposition)
"""
import argparse
import concurrent.futures as cf
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
LLVM = "/opt/rocm/lib/llvm/bin"
HALF_RATE = {"v_alignbit_b32", "v_add3_u32", "v_alignbyte_b32", "v_perm_b32", "v_xad_u32", "v_or3_b32",
             "v_lshl_or_b32", "v_lshl_add_u32", "v_add_lshl_u32", "v_and_or_b32", "v_bfi_b32", "v_bfe_u32",
             "v_mad_u32_u24", "v_pk_add_u16", "v_cndmask_b32_e64"}
COST_A, COST_B, CLOCK = 4.37, 2.66, 2.35e9


def variants():
    out = []
    for ln in open(os.path.join(ROOT, "p1_amd/csrc/fast_variants.inc")):
        m = re.match(r"P1_CASE\((\d+),\s*(\d+),\s*(true|false)\)", ln)
        if m:
            out.append((int(m.group(1)), int(m.group(2)), m.group(3) == "true"))
    return out


def meta(s_text, kern="k_scan"):
    i = s_text.find(f".name:           {kern}\n")
    blk = s_text[i:i + 2000]
    get = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", blk).group(1))
    return {"vgpr": get("vgpr_count"), "sgpr": get("sgpr_count"), "sgpr_spill": get("sgpr_spill_count"),
            "vgpr_spill": get("vgpr_spill_count")}


def loops_of(co, kern="k_scan"):
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True,
                         text=True).stdout.split("\n")
    ins, on = [], False
    for ln in dis:
        mh = re.match(r"^([0-9a-f]+) <(.*)>:", ln)
        if mh:
            on = mh.group(2) == kern
            continue
        m = re.search(r"^\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):\s*((?:[0-9A-Fa-f]{8}\s*)+)(<.*>)?$", ln)
        if on and m:
            ins.append((int(m.group(2), 16), 4 * len(m.group(3).split()), m.group(1)))
    loops = []
    for a, sz, t in ins:
        m = re.match(r"s_cbranch_\w+\s+(\d+)", t)
        if m:
            off = int(m.group(1))
            off = off - 65536 if off >= 32768 else off
            tgt = a + 4 + 4 * off
            if tgt < a:
                loops.append((tgt, a))
    inner = [l for l in loops if not any(o != l and l[0] <= o[0] and o[1] <= l[1] for o in loops)]
    return ins, inner, loops


def parent_of(loop, loops):
    """The smallest loop strictly containing `loop` (None at top level)."""
    outer = [o for o in loops if o != loop and o[0] <= loop[0] and loop[1] <= o[1]]
    return min(outer, key=lambda o: o[1] - o[0]) if outer else None


def mix(ins, lo, hi, exclude=None):
    body = [(a, sz, t) for a, sz, t in ins if lo <= a <= hi and not (exclude and exclude[0] <= a <= exclude[1])]
    A = B = S = other = n8 = at4 = 0
    for a, sz, t in body:
        op = t.split()[0]
        if sz == 8:
            n8 += 1
            at4 += a % 8 == 4
        if op.startswith("v_"):
            if op in HALF_RATE:
                A += 1
            else:
                B += 1
        elif op.startswith("s_"):
            S += 1
        else:
            other += 1
    cyc = A * COST_A + B * COST_B
    return {"valu": A + B, "half_rate_A": A, "full_rate_B": B, "salu": S, "other": other, "bytes": hi - lo + 4,
            "n8": n8, "n8_at_4_mod_8": at4, "pred_simd_cycles_per_wave_iter": cyc,
            "pred_GH_s": 1024 * CLOCK * 64 / cyc / 1e9 if cyc else None}


def build_one(v, waves, isapost):
    fv, nv, tr = v
    with tempfile.TemporaryDirectory() as td:
        inc = os.path.join(td, "v.inc")
        open(inc, "w").write(f"P1_CASE({fv}, {nv}, {'true' if tr else 'false'})\n")
        s = os.path.join(td, "k.s")
        cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-o", s,
               f"-DP1_VARIANTS_INC=\"{inc}\"", os.path.join(ROOT, "p1_amd/csrc/p1hip_kernels.hip")]
        if waves:
            cmd.insert(1, f"-DP1_FAST_WAVES={waves}")
        subprocess.run(cmd, check=True, capture_output=True)
        post = os.path.join(td, "k.post.s")
        subprocess.run([sys.executable, os.path.join(ROOT, "tools/isa_post.py"), s, post] + isapost, check=True,
                       capture_output=True)
        o, co = os.path.join(td, "k.o"), os.path.join(td, "k.co")
        subprocess.run([f"{LLVM}/clang", "-cc1as", "-triple", "amdgcn-amd-amdhsa", "-filetype", "obj", "-target-cpu",
                        "gfx950", "-mrelocation-model", "pic", "-o", o, post], check=True)
        subprocess.run([f"{LLVM}/ld.lld", "-m", "elf64_amdgpu", "--no-undefined", "-shared", "-o", co, o], check=True)
        r = {"variant": [fv, nv, tr]}
        r.update(meta(open(s).read()))
        ins, inner, loops = loops_of(co)
        big = max(inner, key=lambda l: l[1] - l[0])
        r["loop"] = mix(ins, *big)
        # the enclosing loop's own instructions (per trip of it, the inner
        # loop excluded): MODE 7's per-10-nonce block-0 update, the split
        # modes' outer_update
        par = parent_of(big, loops)
        if par:
            r["parent_loop_exclusive"] = mix(ins, par[0], par[1], exclude=big)
        r["waves_per_simd_vgpr"] = min(8, 512 // max(1, r["vgpr"]))
        r["blocks_per_cu_sgpr"] = min(8, 800 // ((-(-r["sgpr"] // 16)) * 16 + 16))
        return r


def explain(paths, ref=(4, 6, False)):
    """per-nonce loop VALU of every 1-block (non-TRAIL)
    digit-update variant against `ref` (c2's 4,6), split into what the lost
    hoisting explains -- each FV step below ref moves one round and one
    schedule word into the loop (the ref family's own per-FV step, read off
    FV, FV+1 of the same mode) and mode 1 vs 6 the wave-uniform word -- and
    the rest, which would be an attributable target."""
    rows = {}
    for p in paths:
        for ln in open(p):
            if ln.startswith("{"):
                d = json.loads(ln)
                rows[tuple(d["variant"])] = d["loop"]
    base = rows[ref]
    # the per-FV step of the ref mode, measured between neighbouring FVs
    steps = {fv: rows[(fv, ref[1], False)]["valu"] - rows[(fv + 1, ref[1], False)]["valu"]
             for fv in range(0, 13) if (fv, ref[1], False) in rows and (fv + 1, ref[1], False) in rows}
    uniform = rows[(ref[0], 1, False)]["valu"] - base["valu"]  # mode 1 vs 6 at the ref FV
    out = []
    for (fv, mode, tr), lp in sorted(rows.items()):
        if tr or mode not in (1, 3, 4, 6) or fv > ref[0] + 2:
            continue
        # split modes 3/4 run the <FV+1, 1> loop per nonce (outer word hoisted)
        efv = fv + 1 if mode in (3, 4) else fv
        lost = sum(steps.get(f, 0) for f in range(efv, ref[0])) - sum(steps.get(f, 0) for f in range(ref[0], efv))
        mode_cost = uniform if mode == 1 else 0  # modes 3/4 keep their inner word uniform too
        d = lp["valu"] - base["valu"]
        out.append({"variant": [fv, mode, tr], "loop_valu": lp["valu"], "A": lp["half_rate_A"],
                    "B": lp["full_rate_B"], "vs_ref": d, "explained_by_fv": lost,
                    "explained_by_uniform_word": mode_cost, "unexplained": d - lost - mode_cost})
    return {"ref": list(ref), "ref_valu": base["valu"], "per_fv_step_valu": steps,
            "mode1_minus_mode6_valu": uniform}, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--explain", nargs="*", default=None,
                    help="read variant report jsonl files and print the FV-floor decomposition instead of building")
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--isapost", default="--no-e64 --align-loops=3 --loop-offset=4 --pair-sched=0 --sched-amax=5 --sched-bmax=4 --prio=0,1")
    a = ap.parse_args()
    if a.explain is not None:
        head, rows = explain(a.explain or [os.path.join(ROOT, "profiles/r03f_variant_report.jsonl")])
        print(json.dumps(head))
        for r in rows:
            print(json.dumps(r))
        return
    vs = variants()
    if a.only:
        want = {tuple(int(x) if x.isdigit() else x == "true" for x in o.split(",")) for o in a.only}
        vs = [v for v in vs if v in want]
    with cf.ThreadPoolExecutor(a.jobs) as ex:
        for r in ex.map(lambda v: build_one(v, a.waves, a.isapost.split()), vs):
            r["waves_build"] = a.waves or 4
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
