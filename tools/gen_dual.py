"""Generate tools/dual.hip: when does gfx950 issue two VALU instructions in
one 4-cycle issue slot?

The c4 PMC pass (profiles/r04g_c4_pmc_summary.json) fits a slot model to
within 1%: SIMD cycles = 4 x (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2), i.e. a
half-rate op (v_alignbit_b32, v_add3_u32) fills a 4-cycle slot, and a
full-rate op fills one too unless a second full-rate op shares it (VALU2).
The scan loop pairs ~56% of its full-rate ops; pairing all of them would
take ~11% off the kernel.  This benchmark finds what a pair needs: the same
wave or any wave, adjacency, independence, encoding size and address parity,
register banks.

Each kernel is one straight-line inline-asm body (>= 240 instructions,
repeated in a scalar loop) over fixed VGPRs; a wave times itself with
s_memtime.  A pattern is a string of instruction kinds (below); the k-th
VALU instruction of the body writes chain register v[40 + k % 16] and reads
it (so it depends on the instruction 16 VALU ops earlier), unless the kind
is followed by '^', which makes it read the previous instruction's result
instead of its first shared source.  Output: one JSON line per (pattern,
alignment, waves/SIMD): SIMD cycles per VALU wave-instruction.
Test tool, not product."""
import os

NCH = 16
BASE = 40          # chain registers v40..v55 (banks 0,1,2,3,0,...)
S1, S2 = 100, 105  # shared sources, banks 0 and 1
SINK = 110         # v_mov destination
KINDS = {
    # half-rate ("A")
    "a": ("v_alignbit_b32 {d}, {d}, {d}, 7", True),
    "c": ("v_add3_u32 {d}, {d}, {s1}, {s2}", True),
    # full-rate, 8-byte VOP3
    "b": ("v_bitop3_b32 {d}, {d}, {s1}, {s2} bitop3:0x96", True),
    "e": ("v_add_u32_e64 {d}, {s1}, {d}", True),
    "x": ("v_xor_b32_e64 {d}, {s1}, {d}", True),
    "l": ("v_lshrrev_b32_e64 {d}, 3, {d}", True),
    "k": ("v_add_u32_e64 {d}, s20, {d}", True),
    # full-rate, 4-byte VOP2
    "d": ("v_add_u32_e32 {d}, {s1}, {d}", True),
    "D": ("v_add_u32_e32 {d}, s20, {d}", True),   # VOP2 with an SGPR source
    "y": ("v_xor_b32_e32 {d}, {s1}, {d}", True),
    "m": ("v_mov_b32_e32 v{sink}, {d}", True),   # reads a chain, writes a sink
    "M": ("v_mov_b32_e32 v{rsink}, {d}", True),  # reads a chain, writes one of 4 sinks in turn
    # scalar fillers
    "n": ("s_nop 0", False),
    "s": ("s_add_u32 s21, s21, 1", False),
    "N": ("s_nop 3", False),
    "H": ("s_setprio 1", False),
    "L": ("s_setprio 0", False),
}

SET1 = [
    # single kinds
    "a", "c", "b", "e", "x", "l", "k", "d", "y",
    # half-rate followed by full-rate runs
    "ad", "ae", "ab", "add", "aee", "abb", "abe", "aadd", "aaee", "aabb", "aabe", "aaadd", "aaaee",
    "addd", "aeee", "adddd", "aeeee",
    # full-rate pairs with one dependent member
    "dd^", "ee^", "bb^", "ad^", "ae^", "add^", "aee^",
    # fillers between the members of a pair
    "dnd", "ene", "dmd", "eme", "ama", "anb",
    # mixed encodings
    "ed", "de", "bd", "db", "aed", "ade", "abd", "adb",
]
# round 2 (r05e): (pattern, alignments mod 32, waves per SIMD)
SET2 = [(p, (0, 4, 8, 12, 16, 20, 24, 28), (4,)) for p in ("aeee", "ae", "b", "aee")] + \
       [(p, (0, 4), (2, 3, 4)) for p in ("ad", "ae", "aee", "aeee", "anb", "ama", "aMa", "asb", "aNb", "b", "d")] + \
       [(p, (4,), (4,)) for p in ("aMaM", "amam", "anbb", "anbbb", "aanbb", "aaanbb", "annb", "abnb", "anbnb", "asbsb",
                                   "adn", "and", "ansd", "aNbb", "aaNbb", "aaabb", "aaNbNb")]
# round 3 (r05k): wave priorities.  Static: a wave's priority from its
# block's slot on the CU (blocks b, b+CUs, b+2 CUs, b+3 CUs share a CU):
# "/2" = half the waves at 1, "/4" = 0..3.  Dynamic: H / L tokens.
SET3 = [(p, (4,), (4,)) for p in ("a", "b", "d", "ae", "aee", "ad", "aaee", "a/2", "b/2", "d/2", "ae/2", "aee/2",
                                    "ad/2", "aaee/2", "a/4", "ae/4", "ad/4", "HaLe", "HaLee", "HaaLee", "HaLeee",
                                    "HaaLe", "HaaaLee", "HaLd", "HaLdd", "LaHe", "HaHe", "HaaaLe", "HaaaaLe")]
# round 4 (r05m): SGPR sources under per-run priorities
SET4 = [(p, (4,), (4,)) for p in ("D", "k", "HaLD", "HaLk", "HkLe", "HcLe", "HaLDD", "HaLkk", "HkLD", "HaLb",
                                    "HaLbb", "HaaLbb", "HaaLbbb", "HaaaLbbbb", "HaLee", "HcLd")]
# round 5 (r05q): can a half-rate op be the second of a slot?  Loop-like A:B mixes
SET5 = [(p, (4,), (4,)) for p in ("HaLa", "HaLc", "HcLa", "HaaLaa", "HaLaa", "HaaLb", "HaaLbHaLbb", "HaaLbHaaLbHaLbb",
                                    "HaaaLbb", "HaaaaLbbb", "HaaaaaaaLbbbbb", "HaLbHaaLb", "HaaLa", "LaHa")]
SET = os.environ.get("DUAL_SET", "1")
if SET == "1":
    RUNS = [(p, (0, 4), (1, 4)) for p in SET1]
elif SET == "2":
    RUNS = SET2
elif SET == "3":
    RUNS = SET3
elif SET == "4":
    RUNS = SET4
else:
    RUNS = SET5
BODY_MIN = 240


def expand(pat):
    toks = []
    i = 0
    while i < len(pat):
        k = pat[i]
        dep = i + 1 < len(pat) and pat[i + 1] == "^"
        toks.append((k, dep))
        i += 2 if dep else 1
    return toks


def body(pat):
    toks = expand(pat)
    nchain = sum(1 for k, _ in toks if k not in "mMnsNHL")
    reps = 1
    while len(toks) * reps < BODY_MIN or (nchain * reps) % NCH:
        reps += 1
    lines, v, prev, r = [], 0, None, 0
    for _ in range(reps):
        for k, dep in toks:
            tmpl, counts = KINDS[k]
            d = f"v{BASE + v % NCH}"
            s1 = prev if (dep and prev) else f"v{S1}"
            lines.append(tmpl.format(d=d, s1=s1, s2=f"v{S2}", sink=SINK, rsink=SINK + r % 4))
            if k == "M":
                r += 1
            if k not in "mMnsNHL":
                prev = d
                v += 1
    n_valu = sum(1 for k, _ in toks if k not in "nsNHL") * reps
    return lines, n_valu


CLOB = ",".join(f'"v{BASE + i}"' for i in range(NCH)) + f',"v{S1}","v{S2}","s20","s21",' + \
    ",".join(f'"v{SINK + i}"' for i in range(4))

out = ["// GENERATED by tools/gen_dual.py -- do not edit.  Test tool, not product.",
       "#include <hip/hip_runtime.h>", "#include <stdint.h>", "#include <stdio.h>", "",
       '#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\\n", #x, hipGetErrorString(e)); return 1; } } while (0)',
       ""]
init = "\\n\\t".join([f"v_mov_b32 v{BASE + i}, %[s]" for i in range(NCH)] +
                     [f"v_mov_b32 v{S1}, %[s]", f"v_mov_b32 v{S2}, %[s]", f"v_mov_b32 v{SINK}, 0",
                      "s_mov_b32 s20, 12345", "s_mov_b32 s21, 0"])
kernels = []
for pat, aligns, wlist in RUNS:
    pat, _, static = pat.partition("/")
    lines, nvalu = body(pat)
    prio = ""
    if static:
        prio = (f"  const int slot = (int)(blockIdx.x / gridDim.x * 0 + blockIdx.x / (gridDim.x / {wlist[0]}));\n"
                f"  if (slot % {static} == 1) __builtin_amdgcn_s_setprio(1);\n"
                f"  if (slot % {static} == 2) __builtin_amdgcn_s_setprio(2);\n"
                f"  if (slot % {static} == 3) __builtin_amdgcn_s_setprio(3);\n")
        pat = pat + "/" + static
    for al in aligns:
        i = len(kernels)
        pre = ".p2align 6" + "\\n\\ts_nop 0" * (al // 4)
        asm = "\\n\\t".join(lines)
        out.append(f"""__global__ __launch_bounds__(256) void k{i}(uint64_t* out, uint32_t seed, int iters) {{
  asm volatile("{init}" : : [s] "v"(seed * (threadIdx.x + 1)) : {CLOB});
{prio}  int cnt = iters;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile("{pre}\\n1:\\n\\t{asm}\\n\\ts_sub_u32 %[c], %[c], 1\\n\\ts_cmp_lg_u32 %[c], 0\\n\\ts_cbranch_scc1 1b"
               : [c] "+s"(cnt) : : "scc", {CLOB});
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t keep;
  asm volatile("v_mov_b32 %0, v{BASE}" : "=v"(keep));
  if (threadIdx.x % 64 == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = (t1 - t0) + (keep == 0x7fffffffu ? 1 : 0);
}}""")
        kernels.append((f"k{i}", pat, al, nvalu, wlist))

out.append("""template <typename K>
static int run(K kern, const char* pat, int al, int nvalu, int cus, uint64_t* d, uint64_t* h, int w0, int w1, int w2) {
  const int iters = 1024;
  for (int wps : {w0, w1, w2}) {
    if (wps == 0) continue;
    const int blocks = cus * wps;  // 4 waves per block, one per SIMD
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d, 1u + rep, iters);
      CHK(hipDeviceSynchronize());
    }
    CHK(hipMemcpy(h, d, sizeof(uint64_t) * blocks * 4, hipMemcpyDeviceToHost));
    double sum = 0, mx = 0;
    for (int i = 0; i < blocks * 4; ++i) { sum += (double)h[i]; if ((double)h[i] > mx) mx = (double)h[i]; }
    const double winst = (double)iters * nvalu;
    printf("{\\"pattern\\": \\"%s\\", \\"align\\": %d, \\"waves_per_simd\\": %d, \\"valu_per_body\\": %d, "
           "\\"simd_cyc_per_valu\\": %.3f, \\"max\\": %.3f}\\n",
           pat, al, wps, nvalu, sum / (blocks * 4) / winst / wps, mx / winst / wps);
    fflush(stdout);
  }
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  if (cus > 256) return 2;
  printf("{\\"device\\": \\"%s\\", \\"cus\\": %d, \\"clock_khz\\": %d}\\n", p.gcnArchName, cus, p.clockRate);
  uint64_t* d;
  CHK(hipMalloc(&d, sizeof(uint64_t) * 256 * 4 * 4));
  static uint64_t h[256 * 4 * 4];""")
for name, pat, al, nvalu, wl in kernels:
    w = list(wl) + [0] * (3 - len(wl))
    out.append(f'  if (run({name}, "{pat}", {al}, {nvalu}, cus, d, h, {w[0]}, {w[1]}, {w[2]})) return 1;')
out.append("  CHK(hipFree(d));\n  return 0;\n}")
open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "dual.hip" if SET == "1" else f"dual{SET}.hip"), "w").write("\n".join(out) + "\n")
print(len(kernels), "kernels")
