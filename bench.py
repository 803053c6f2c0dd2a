#!/usr/bin/env python3
"""bench.py -- nonce-scan throughput of libp1hip.so on MI355X.

Metric (BASELINE.json): SHA-256 nonce-hashes/s (GH/s) at 1/2/4/8 MI355X and
the fraction of the integer-VALU roofline.

Workloads (BASELINE.json configs):
  c4  configs[3]: msg "bradfitz", the FIXED job [0, 2^38) split contiguously
      over the N GPUs (strong scaling).  The default at EVERY N: north_star's
      1 -> 8 GPU scaling target is stated on this range, so the N = 1 line
      and every point of the driver's 1/2/4/8 scaling run time the same job.
  c2  configs[1]: msg "bradfitz" (8 B), nonces [0, 2^32) per GPU, one SHA-256
      compression per nonce.
  c3  configs[2]: 120-byte msg (host midstate), [0, 2^34) per GPU, 2 tail blocks.
At N = 1 the line also carries c2 and c3 as timed sub-results (`by_config`),
each checked against its independently pinned answer.
A step is one full scan of the job (the drop-in for miner.go:56-63) ending
with the (hash, nonce) result on the host.

Production settings only: the library's test knobs (P1HIP_*, honoured only
under P1HIP_TEST_KNOBS=1) must be off -- bench.py exits 4 before timing
anything otherwise, and prints "test_knobs": {} in the line.

How N GPUs are driven:
  * torchrun (WORLD_SIZE > 1, the driver's launch): one process per GPU; each
    rank scans one contiguous shard through the library and the 16-byte
    results are all-gathered over torch.distributed "nccl" (RCCL over xGMI).
  * `python bench.py --gpus N` without torchrun: ONE process opens N devices
    through the library itself (p1hip_init(N): one host thread per device,
    ncclCommInitAll, ncclAllGather of the 16-byte partials inside p1hip_scan).
  * --gpus larger than the visible device count exits non-zero; it never
    silently falls back to fewer GPUs.

Prints ONE JSON line on rank 0.
"""
import argparse
import glob
import json
import os
import re
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# int32 VALU peak of one MI355X: 256 CUs x 4 SIMD x 32 lanes (wave64 VALU op
# issues in 2 cycles on CDNA4's SIMD-32, MI355X_MICROARCH.md "Execution model")
# x 2.4 GHz max clock.  tools/valu_peak measures the per-instruction rates
# (profiles/r01_valu_peak.jsonl).
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9
# (SURVEY.md 8(d)'s 39.32 T/s assumed 64 lane-ops/clk/CU; it is superseded by
# this figure, which tools/valu_peak confirms for add/xor/shift/bitop3 --
# DESIGN.md 4 "Roofline numbers".)
ALG_OPS_PER_COMPRESSION = 1384  # 64 rounds x 14 + 48 schedule words x 10 + 8
# The reference's own published rate for bitcoin.Hash: "around 10,000 per
# second" on a typical Andrew Linux machine (p1.pdf 4.1).
PUBLISHED_HASHES_PER_S = 1.0e4

CONFIGS = {
    "c2": {"msg": b"bradfitz", "per_gpu": 1 << 32, "b_tail": 1,
           "desc": "configs[1]: 8-byte msg 'bradfitz', nonces [0,2^32) per GPU, 1 SHA-256 block/nonce"},
    "c3": {"msg": b"cmu440-p1-" * 12, "per_gpu": 1 << 34, "b_tail": 2,
           "desc": "configs[2]: 120-byte msg, host midstate, nonces [0,2^34) per GPU, 2 tail blocks/nonce"},
    # configs[3]: the fixed 2^38 job split over however many GPUs run (strong scaling)
    "c4": {"msg": b"bradfitz", "total": 1 << 38, "b_tail": 1,
           "desc": "configs[3]: 8-byte msg 'bradfitz', nonces [0,2^38) split contiguously over the GPUs"},
}
GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.json")


# The algorithmic SHA-256 compression (SURVEY.md 8(d)'s 1384 ops) by
# instruction class: 64 rounds x (6 rotr, 4 bitop3, 3 add3, 1 add) +
# 48 schedule words x (4 rotr, 2 shr, 2 bitop3, 1 add3, 1 add) + 8 adds.
ALG_MIX = {"v_alignbit_b32": 576, "v_bitop3_b32": 352, "v_add3_u32": 240, "v_add_u32": 120,
           "v_lshrrev_b32": 96}
VALU_PEAK_PROFILE = "profiles/r01_valu_peak.jsonl"
# Per-variant loop mix of the shipped kernel (tools/variant_report.py run
# through the shipped post-pass on the round-6 work-queue k_scan: all 78
# variants; VALU counts identical to the r02d/r02k/r03f reports and to the
# static-grid r06 report except 0,3 / 0,4 at 3 fewer): A "half-rate" ops (v_alignbit_b32, v_add3_u32, ...)
# and B full-rate ops per nonce.  A SIMD issues VALU ops in 4-cycle slots; an
# A op only as the first op of a slot, a B op also as the second (another
# wave's), so a loop cannot issue in fewer than 4 x max(A, (A + B) / 2)
# SIMD cycles per 64 nonces (DESIGN.md 4 "Dual issue", tools/gen_dual.py).
VARIANT_PROFILES = ["profiles/r06d_variant_report.jsonl"]
VARIANT_PROFILE = ", ".join(VARIANT_PROFILES)
SLOT_CYCLES = 4.0  # SIMD cycles per VALU issue slot (gfx950; DESIGN.md 4 "Dual issue")


class UsageError(SystemExit):
    pass


def resolve_run(gpus, config, env, visible, force_dist=False):
    """How this invocation uses the GPUs.

    Returns a dict: mode ("single" | "library" | "torchrun"), n (GPUs in the
    job), rank, world (processes), local_rank, config.  Raises UsageError
    (non-zero exit) when the request cannot be honoured -- never falls back to
    fewer GPUs than asked for.  force_dist (--dist) takes the torchrun path
    even for a world of one process, to rehearse it on a one-GPU box."""
    world = int(env.get("WORLD_SIZE", "1") or 1)
    rank = int(env.get("RANK", "0") or 0)
    local = int(env.get("LOCAL_RANK", "0") or 0)
    if gpus < 1:
        raise UsageError(f"bench.py: --gpus must be >= 1 (got {gpus})")
    if world > 1 or force_dist:
        if gpus != world:
            raise UsageError(f"bench.py: --gpus {gpus} but torchrun started {world} ranks (WORLD_SIZE)")
        mode, n = "torchrun", world
    else:
        if gpus > visible:
            raise UsageError(f"bench.py: --gpus {gpus} but only {visible} GPU(s) are visible")
        mode, n = ("library" if gpus > 1 else "single"), gpus
    cfg = config or "c4"  # north_star's scaling job at every N
    return {"mode": mode, "n": n, "rank": rank, "world": world, "local_rank": local, "config": cfg}


def job_total(cfg, n):
    return cfg["total"] if "total" in cfg else cfg["per_gpu"] * n


def layout_config(spec):
    """--layout L,START[,N]: a measurement job outside BASELINE's configs --
    tools/sweep.py's L-byte message, nonces [START, START + N) (N default
    2^32) -- to profile one tail layout (the two-block
    TRAIL loops).  Same kernel path as every scan; no pinned answer."""
    parts = [int(x, 0) for x in spec.split(",")]
    if len(parts) not in (2, 3) or parts[0] < 0 or parts[1] < 0:
        raise UsageError(f"bench.py: --layout L,START[,N], got {spec!r}")
    L, start = parts[0], parts[1]
    n = parts[2] if len(parts) == 3 else 1 << 32
    d = len(str(start))
    if len(str(start + n - 1)) != d:
        raise UsageError("bench.py: --layout range must stay inside one decade (one kernel variant)")
    b_tail = 1 if (L + 1) % 64 + d + 9 <= 64 else 2
    msg = bytes((33 + (i * 7) % 90) for i in range(L))
    return {"msg": msg, "total": n, "lo": start, "hi": start + n - 1, "b_tail": b_tail, "layout": [L, d],
            "variant": list(fast_variant(L, d)),
            "desc": f"layout L={L} d={d} (tools/sweep.py message, variant {list(fast_variant(L, d))}), "
                    f"nonces [{start}, {start + n}) on each run"}


def known_answer(cfg, n):
    """The exact answer of this job when one is pinned independently of the
    GPU: tests/golden/golden.json's large vectors (configs[1]: the survey's
    hashlib run; configs[2], [3]: tools/pin_large.c, a CPU restatement
    validated against the oracle and hashlib).  Returns ((hash, nonce),
    source) or (None, None)."""
    total = job_total(cfg, n)
    try:
        with open(GOLDEN) as f:
            vecs = json.load(f)["scan"]
    except (OSError, ValueError, KeyError):
        return None, None
    if "lo" in cfg:
        return None, None
    for v in vecs:
        if v.get("large") and bytes.fromhex(v["msg_hex"]) == cfg["msg"] and v["lower"] == 0 \
                and v["upper"] == total - 1:
            src = v["source"]
            if v.get("reference_pinned") is False:
                src += " [parity-unpinned: no reference-held fixture covers this range]"
            return (v["hash"], v["nonce"]), src
    return None, None


def mix_roofline():
    """Hashes/s one MI355X would reach if every instruction of the
    algorithmic compression issued at its own measured peak rate
    (tools/valu_peak, 8 waves/SIMD, lane-ops/clk/CU) at 2.4 GHz."""
    path = os.path.join(ROOT, VALU_PEAK_PROFILE)
    if not os.path.exists(path):
        return None
    rate = {}
    names = {"v_alignbit_b32 (x,x,imm)": "v_alignbit_b32", "v_bitop3_b32 0x96": "v_bitop3_b32",
             "v_add3_u32": "v_add3_u32", "v_add_u32_e32": "v_add_u32", "v_lshrrev_b32_e32": "v_lshrrev_b32"}
    with open(path) as f:
        for line in f:
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            if d.get("instr") in names and d.get("blocks_per_cu_wave_slots") == 8:
                rate[names[d["instr"]]] = d["per_cu_per_clk_at_2.4GHz"]
    if set(rate) != set(ALG_MIX):
        return None
    cu_cycles = sum(n / rate[k] for k, n in ALG_MIX.items())  # per nonce per compression
    return {"peak_GH_s_per_block": 256 * 2.4e9 / cu_cycles / 1e9, "cu_cycles_per_compression": cu_cycles,
            "rates_lane_ops_per_clk_cu": rate, "source": VALU_PEAK_PROFILE}


def fast_variant(msg_len, d, k=3):
    """(FV, MODE, TRAIL) the planner picks for a d-digit decade of a message
    of msg_len bytes at lo-digit count k (planner.hpp make_layout/add_fast;
    MODE as in scan_core.hpp fast_thread: 1 = lo digits in one word, 3/4 =
    straddling lo digits split with the hundreds / hundreds and tens in the
    outer word, 5 = tail block 1 holds only lo digits, its schedule tabulated)."""
    r = (msg_len + 1) % 64
    q = r + d - 1
    nb = 1 if r + d + 9 <= 64 else 2
    if nb == 1:
        vb, trail = 0, False
    elif q <= 63:
        vb, trail = 0, True
    elif q == 64 and d > 3:
        return 15, 7, False  # MODE 7: units alone in tail block 1 (table), tens/hundreds in block 0's W15
    elif q - 63 <= 7:
        return 0, 5, False  # MODE 5: tail block 1 holds only the lo digits (k = q - 63)
    else:
        vb, trail = 1, False
    qv = q - 64 * vb
    fv = (qv - k + 1) >> 2
    if (qv >> 2) == fv:
        # 6 = mode 1 with the lo digits from byte 0 of word FV (a wave-uniform word)
        return fv, 6 if (qv - k + 1) % 4 == 0 and not trail else 1, trail
    return fv, 4 if k >= 2 and ((qv - 1) >> 2) == fv else 3, trail


def workload_mix(msg_len, lo, hi):
    """Nonce-weighted loop mix (half-rate A, full-rate B VALU instructions per
    nonce) of the fast variants that scan [lo, hi]."""
    table = {}
    for rel in VARIANT_PROFILES:
        path = os.path.join(ROOT, rel)
        if not os.path.exists(path):
            return None
        for line in open(path):
            if line.startswith("{"):
                d = json.loads(line)
                loop = dict(d["loop"])
                par = d.get("parent_loop_exclusive")
                if d["variant"][1] == 7 and par:  # MODE 7: + block 0's update, once per 10 nonces
                    loop["half_rate_A"] += par["half_rate_A"] / 10
                    loop["full_rate_B"] += par["full_rate_B"] / 10
                table[tuple(d["variant"])] = loop
    a = b = w = 0.0
    for d in range(1, 21):
        dlo, dhi = (0 if d == 1 else 10 ** (d - 1)), 10 ** d - 1
        n = min(hi, dhi) - max(lo, dlo) + 1
        if n <= 0 or d <= 3:
            continue
        v = table.get(fast_variant(msg_len, d))
        if v is None:
            return None
        a += n * v["half_rate_A"]
        b += n * v["full_rate_B"]
        w += n
    return (a / w, b / w) if w else None


def profile_tag_key(path):
    """Session order of a profiles/ file: round number, then the session
    letters by length and then alphabet (r05z < r05aa < r05ag), so "newest"
    is not an accident of lexical sorting."""
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")


def pmc_summary(config, codeobj):
    """The committed rocprofv3 PMC summary of this config's k_scan launches
    that was taken on THIS code object: profiles/*_pmc_summary.json written
    by tools/summarize_prof.py carry the codeobj_sha256 of the library the
    profiled command loaded (the counters come from separate --pmc passes of
    the same bench command).  Newest session among the matches; (None,
    None) when no summary was taken on this build."""
    best = None
    for p in glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")):
        with open(p) as f:
            d = json.load(f)
        if d.get("config", "c2") != config or not codeobj or d.get("codeobj_sha256") != codeobj:
            continue
        if best is None or profile_tag_key(p) > profile_tag_key(best[1]):
            best = (d, p)
    return (best[0], os.path.relpath(best[1], ROOT)) if best else (None, None)


def host_cores():
    """CPU cores this process may run on: the affinity mask, capped by the
    cgroup CPU quota when one is set (a GPU box shares its host)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return (min(n, quota) if quota else n), n, quota, model


def cpu_baseline(msg, start, target_s, runs=5):
    """Oracle restatement (format + full SHA-256 per nonce, the reference's
    per-nonce work) on every host core this process may use, contiguous
    sub-ranges per thread (the reference's goroutine-per-core plan,
    BASELINE.md 4); median of `runs` timed runs over a bounded sample."""
    import oracle

    threads, affinity, quota, model = host_cores()
    cal = 1 << 16
    t0 = time.perf_counter()
    oracle.scan(msg, start, start + cal * threads - 1, threads=threads)
    rate = cal * threads / (time.perf_counter() - t0)
    n = max(int(rate * target_s / runs), cal * threads)
    rates = []
    for i in range(runs):
        lo = start + i * n
        t0 = time.perf_counter()
        oracle.scan(msg, lo, lo + n - 1, threads=threads)
        rates.append(n / (time.perf_counter() - t0))
    med = statistics.median(rates)
    return {
        "value": med / 1e9,
        "unit": "GH/s",
        "cores": threads,
        "kind": "port",
        "runs_GH_s": [r / 1e9 for r in rates],
        "host": {"cpu_model": model, "affinity_cpus": affinity, "cgroup_quota_cpus": quota,
                 "os_cpu_count": os.cpu_count()},
        "sample": f"oracle/p1_oracle.c (C restatement of hash.go:13-17 + miner.go:56-63: %d formatting + "
                  f"full SHA-256 per nonce; not the Go reference, which cannot be built here), {threads} "
                  f"threads over contiguous sub-ranges, median of {runs} runs of {n} nonces each starting "
                  f"at nonce {start} of the same message",
    }


def scaling_report(units, steps, ms_per_step):
    """Per-GPU accounting of a timed run (one entry per rank under torchrun,
    per device in library mode), so an N > 1 line explains its own scaling:
    a straggler shard shows as kernel_ms_max_over_mean > 1, a slow exchange
    as gather_ms_per_step, launch/host skew as step time not covered by the
    slowest GPU's kernels.  Each unit: shard_lo/shard_hi (lo > hi: empty),
    nonces, launches, alg_ops, kernel_ms, scan_ms, gather_ms (sums over the
    timed steps)."""
    out = []
    for u in units:
        k = u["kernel_ms"]
        e = {"unit": u.get("rank", u.get("device")),
             "shard": [u["shard_lo"], u["shard_hi"]] if u["shard_lo"] <= u["shard_hi"] else None,
             "nonces_per_step": u["nonces"] / steps,
             "launches_per_step": u["launches"] / steps,
             "kernel_ms_per_step": k / steps,
             "scan_ms_per_step": u["scan_ms"] / steps,
             "gather_ms_per_step": u["gather_ms"] / steps,
             "frac": (u["alg_ops"] / (k * 1e-3) / VALU_PEAK_OPS) if k > 0 else None,
             "kernel_GH_s": (u["nonces"] / (k * 1e-3) / 1e9) if k > 0 else None}
        if "ordinal" in u:
            e["ordinal"] = u["ordinal"]
        if "identity" in u:
            e["identity"] = u["identity"]
        for k in ("rccl_ranks", "rccl_rank"):
            if k in u:
                e[k] = u[k]
        out.append(e)
    ks = [e["kernel_ms_per_step"] for e in out if e["shard"] is not None]
    rep = {"units": out}
    if ks and max(ks) > 0:
        mean = sum(ks) / len(ks)
        slow = max(range(len(out)), key=lambda i: out[i]["kernel_ms_per_step"])
        rep.update({
            "kernel_ms_max_over_mean": max(ks) / mean,
            "slowest_unit": out[slow]["unit"],
            "slowest_kernel_ms_per_step": max(ks),
            "gather_ms_per_step_max": max(e["gather_ms_per_step"] for e in out),
            # ms_per_step = slowest kernel + everything else (planning, launch,
            # sync, the all-gather, skew between GPUs)
            "step_ms_not_in_slowest_kernel": ms_per_step - max(ks),
            "kernel_share_of_step": max(ks) / ms_per_step if ms_per_step > 0 else None,
        })
    return rep


def rocprof_row(config, codeobj):
    """The committed rocprofv3 summary of this config's timed k_scan
    launches taken on THIS code object (profiles/*_<config>_kernel_stats_
    workload.csv, the row over the launches after the warm-up ones,
    tools/summarize_prof.py --skip-launches; its Codeobj_SHA256 column names
    the code object the profiled command ran).  Newest matching session:
    (average ns per launch, source) or (None, None)."""
    import csv

    best, key = (None, None), None
    for p in glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_kernel_stats_workload.csv")):
        with open(p) as f:
            for row in csv.DictReader(f):
                if not (row["Name"].startswith("k_scan (launches after") and codeobj
                        and row.get("Codeobj_SHA256") == codeobj):
                    continue
                if key is None or profile_tag_key(p) > key:
                    best, key = (float(row["AverageNs"]), os.path.relpath(p, ROOT)), profile_tag_key(p)
    return best


class RooflineError(ValueError):
    pass


def check_work_bound(roof):
    """Refuse a line whose kernel could not have done the work it is charged
    with.  The algorithmic `frac` is a speed ratio,
    not a utilisation: the kernel hoists rounds 0..FV-1 and the constant
    schedule words, so a fast layout legitimately exceeds 1 (the r05af
    sweep's [13,6] layouts: 1.052).  The bound is on instructions the kernel
    must execute instead, and either of these above 1 raises RooflineError:
      * executed.frac = PMC VALU lane-instructions per nonce (this code
        object's summary) x this run's kernel rate / peak;
      * work_bound.frac = the per-nonce loop VALU of the variants this
        workload runs (tools/variant_report.py: the loop alone, a floor on
        what a nonce executes) x this run's kernel rate / peak."""
    for path, d in (("roofline.executed", roof.get("executed")), ("roofline.work_bound", roof.get("work_bound"))):
        v = d.get("frac") if isinstance(d, dict) else None
        if isinstance(v, (int, float)) and v > 1.0:
            raise RooflineError(f"{path}.frac = {v:.4f} > 1: the kernel rate exceeds what its own instruction "
                                f"count allows at the {VALU_PEAK_OPS / 1e12:.2f} T peak")


def clock_from_stamps(before, after, wall_hz):
    """Average shader clock of each XCC between two clock-probe stamps
    (tools/clock_probe.hip): the s_memtime midpoint delta over the
    s_memrealtime delta x the wall-counter rate.  before / after: one
    (memtime, memrealtime, memtime, xcc) per workgroup; the first workgroup
    seen on each XCC is its sample.  None when no XCC pairs up."""
    def first(stamps):
        out = {}
        for t0, r, t1, x in stamps:
            out.setdefault(int(x), ((t0 + t1) / 2.0, r))
        return out

    b, a = first(before), first(after)
    per, span = {}, []
    for x in sorted(set(a) & set(b)):
        dt, dr = a[x][0] - b[x][0], a[x][1] - b[x][1]
        if dt > 0 and dr > 0:
            per[x] = dt * wall_hz / dr / 1e9
            span.append(dr / wall_hz)
    if not per:
        return None
    v = list(per.values())
    return {"mean_GHz": sum(v) / len(v), "min_GHz": min(v), "max_GHz": max(v),
            "per_xcc_GHz": {str(k): per[k] for k in per}, "interval_s": max(span)}


CLOCK_PROBE_LIB = os.path.join(ROOT, "tools", "libp1clock.so")


class ClockProbe:
    """Shader-clock stamps of every XCD of the given devices
    (tools/libp1clock.so, tools/clock_probe.hip), taken just outside the
    timed steps on a stream of its own: the timed kernels are untouched.
    Measurement only: without the library the line reports no clock and
    says why."""
    NBLOCKS = 64  # workgroups per stamp: 8 per XCD under round-robin dispatch

    def __init__(self, devices, path=CLOCK_PROBE_LIB):
        import ctypes

        self.devices, self.lib, self.error = list(devices), None, None
        if not os.path.exists(path):
            self.error = f"{os.path.relpath(path, ROOT)} not built"
            return
        lib = ctypes.CDLL(path)
        lib.p1clk_stamp.restype = ctypes.c_int
        lib.p1clk_stamp.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong)]
        lib.p1clk_wall_rate_khz.restype = ctypes.c_int
        lib.p1clk_wall_rate_khz.argtypes = [ctypes.c_int]
        self.lib = lib

    def stamp(self):
        """{device: [(memtime, memrealtime, memtime, xcc)] per workgroup} or None"""
        import ctypes

        if self.lib is None:
            return None
        out = {}
        for d in self.devices:
            buf = (ctypes.c_ulonglong * (4 * self.NBLOCKS))()
            rc = self.lib.p1clk_stamp(d, self.NBLOCKS, buf)
            if rc != 0:
                self.error = f"p1clk_stamp(device {d}) returned hipError {rc}"
                return None
            out[d] = [tuple(buf[4 * i:4 * i + 4]) for i in range(self.NBLOCKS)]
        return out

    def clock(self, before, after):
        """The `clock` record of the interval between two stamps."""
        if before is None or after is None:
            return {"effective_clock_GHz": None, "error": self.error or "no stamps"}
        devs = {}
        for d in self.devices:
            khz = self.lib.p1clk_wall_rate_khz(d)
            c = clock_from_stamps(before.get(d, []), after.get(d, []), khz * 1e3) if khz > 0 else None
            devs[str(d)] = dict(c, wall_counter_kHz=khz) if c else {"error": f"no XCC pairs (wall {khz} kHz)"}
        means = [c["mean_GHz"] for c in devs.values() if "mean_GHz" in c]
        ghz = sum(means) / len(means) if means else None
        rec = {"effective_clock_GHz": ghz, "devices": devs,
               "method": "tools/clock_probe.hip stamps before and after the timed steps: delta s_memtime "
                         "(shader cycles) / delta s_memrealtime x its rate, per XCC, mean over XCCs and devices "
                         "(MI355X_MICROARCH.md 'DVFS give-back' item 6)"}
        if ghz is not None and not 0.3 < ghz < 3.0:
            rec["implausible"] = True
        return rec


def assemble_roofline(config, cfg, stats, steps, pmc=None, pmc_src=None, rocprof=(None, None), single_gpu=True,
                      codeobj=None, clock=None):
    """The bench line's `roofline` block for the dominant kernel k_scan.

    achieved = algorithmic ops (1384 x B_tail per nonce) /
    the HIP-event duration of the launches (stats: scan_alg_ops,
    scan_kernel_ms, scan_launches, scan_nonces summed over this process's
    devices); peak = 78.64 T int32 lane-ops/s.  Beside it: frac_rocprof (the
    same ops over the rocprofv3 average of this config's timed launches,
    single GPU only), the executed-instruction fraction from the PMC
    summary and the loop-mix issue fraction -- each from a profile of THIS
    code object (`codeobj`, sha256) or null with profile_stale -- and, with
    `clock` (ClockProbe.clock), the sustained shader clock of the timed
    steps and the fraction of the peak at that clock."""
    k_ms = stats["scan_kernel_ms"]
    k_n = stats["scan_launches"]
    achieved = stats["scan_alg_ops"] / (k_ms * 1e-3) if k_ms > 0 else 0.0
    k_rate = stats["scan_nonces"] / (k_ms * 1e-3) if k_ms > 0 else 0.0  # nonces/s per device
    lo = cfg.get("lo", 0)
    hi = cfg["hi"] if "hi" in cfg else job_total(cfg, 1) - 1
    roof = {
        "bound": "valu-int32",
        "achieved": achieved / 1e12,
        "peak": VALU_PEAK_OPS / 1e12,
        "unit": "TOP/s",
        "frac": achieved / VALU_PEAK_OPS,
        "frac_kind": "algorithmic ops (SURVEY.md 8(d)) per second / peak: a speed ratio, not a utilisation -- "
                     "hoisting lets a layout exceed 1; the work bound is `work_bound` / `executed`",
        "peak_basis": "256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md; tools/valu_peak); "
                      "supersedes SURVEY.md 8(d)'s 39.32 T",
        "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
        "traffic_unit": "bytes/launch (PMC FETCH_SIZE+WRITE_SIZE)",
        "traffic_source": pmc_src,
        "kernel": "k_scan (one launch per scan covers every decade; algorithmic ops = 1384 x B_tail per nonce)",
        "alg_ops_per_nonce": ALG_OPS_PER_COMPRESSION * cfg["b_tail"],
        "avg_launch_ms": k_ms / k_n if k_n else None,
        "launches_per_step": k_n / steps if steps else None,
        "kernel_hashes_per_s_G": k_rate / 1e9,
        "fast_nonce_share": stats["fast_nonces"] / max(1, stats["fast_nonces"] + stats["generic_nonces"]),
        "codeobj_sha256": codeobj,
    }
    line_clk = clock.get("effective_clock_GHz") if clock and not clock.get("implausible") else None
    if clock is not None:
        roof["clock"] = clock
        roof["effective_clock_GHz"] = line_clk
        if line_clk:
            # the same algorithmic rate against the peak at the clock the
            # chip actually sustained over the timed steps (DVFS)
            roof["frac_at_sustained_clock"] = achieved / (VALU_PEAK_OPS * line_clk / 2.4)
    if pmc and pmc.get("write_bytes_per_launch_calibrated") is not None:
        # WRITE_SIZE counts k_scan's 16-B-per-workgroup partial stores 2x
        # (profiles/r04c_wcal.json): the calibrated bytes against the
        # algorithmic ones (16 B per workgroup)
        roof["traffic_calibrated"] = pmc["write_bytes_per_launch_calibrated"] + pmc.get("fetch_bytes_per_launch", 0.0)
        roof["alg_bytes_per_launch"] = pmc.get("partials_bytes_per_launch")
        roof["traffic_note"] = pmc.get("traffic_note")
    avg_ns, src = rocprof
    stale = []
    if single_gpu:
        roof["frac_rocprof"] = None
        roof["rocprof_source"] = src
        if avg_ns and k_n:
            # one launch of this config's plan; rocprofv3 --kernel-trace
            # average of the same command's timed launches, same code object
            roof["frac_rocprof"] = stats["scan_alg_ops"] / k_n / (avg_ns * 1e-9) / VALU_PEAK_OPS
            roof["rocprof_avg_launch_ms"] = avg_ns / 1e6
            tr = (pmc or {}).get("trace_run") or {}
            if tr.get("effective_clock_GHz"):
                # the clock the traced command ran at (its own probe), so a
                # gap between this run and the trace reads as clock or not
                roof["rocprof_clock_GHz"] = tr["effective_clock_GHz"]
        else:
            stale.append("rocprof")
    roof["executed"] = None
    if not pmc:
        stale.append("pmc")
    elif pmc.get("valu_wave_instr_per_nonce"):
        # SURVEY.md 8(d) accounting rule: the executed-instruction fraction
        # SQ_INSTS_VALU x 64 / (t x peak), this run's kernel rate x the PMC
        # instructions per nonce
        ipn = pmc["valu_wave_instr_per_nonce"]
        ex = {
            "valu_instr_per_nonce": ipn,
            "achieved": ipn * k_rate / 1e12,
            "frac": ipn * k_rate / VALU_PEAK_OPS,
            "simd_cycles_per_valu_wave_instr": pmc.get("simd_cycles_per_valu_wave_instr"),
            "effective_clock_GHz": pmc.get("effective_clock_GHz"),
            "source": pmc_src,
            "note": "frac counts executed VALU lane-instructions against the same 78.6 T peak "
                    "(SURVEY.md 8(d) accounting rule)",
        }
        if line_clk:
            ex["frac_at_sustained_clock"] = ex["frac"] * 2.4 / line_clk
        mix_ab = workload_mix(len(cfg["msg"]), lo, hi)
        if mix_ab and k_rate > 0:
            # the executed loop mix at its ideal issue rate vs the SIMD
            # cycles this run spent per wave-iteration (64 nonces), at this
            # run's own clock when the probe measured it
            clk = (line_clk or pmc.get("effective_clock_GHz") or 2.4) * 1e9
            spent = 1024 * clk * 64 / k_rate
            # DESIGN.md 4 "Dual issue": one VALU issue slot per SIMD per
            # SLOT_CYCLES; a half-rate op issues only as the first op of a
            # slot, a full-rate op may be the second (another wave's), so a
            # loop of A half-rate and B full-rate ops needs at least
            # max(A, (A + B) / 2) slots
            ideal = SLOT_CYCLES * max(mix_ab[0], (mix_ab[0] + mix_ab[1]) / 2.0)
            ex["mix_issue_frac"] = ideal / spent
            ex["mix_issue_clock"] = "this run (clock probe)" if line_clk else "PMC session"
            ex["loop_mix_per_nonce"] = {"half_rate_A": mix_ab[0], "full_rate_B": mix_ab[1],
                                        "source": VARIANT_PROFILE}
            ex["mix_issue_note"] = ("fewest SIMD cycles the loop mix can issue in (4 x max(A, (A + B) / 2): "
                                    "a half-rate op takes a 4-cycle slot as its first op, a full-rate op of "
                                    "another wave may share it; tools/dual*, DESIGN.md 4 'Dual issue') / SIMD "
                                    "cycles spent per 64 nonces")
            v2 = pmc.get("dual_valu_issue_quads_per_wave_instr")
            if v2 is not None:
                # DESIGN.md 4 "Dual issue": one VALU slot per 4 cycles; its
                # first op of any class, a second full-rate op of another
                # wave beside it (SQ_ACTIVE_INST_VALU2)
                n_ab = mix_ab[0] + mix_ab[1]
                ex["dual_issue"] = {"valu2_per_valu": v2, "valu_ops_in_shared_slots": 2.0 * v2,
                                    "shared_slot_bound": 2.0 * min(mix_ab[1], n_ab / 2.0) / n_ab,
                                    "slot_model_simd_cycles_per_valu": 4.0 * (1.0 - v2),
                                    "source": pmc_src,
                                    "note": "SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU from the PMC summary; a slot holds "
                                            "one op of any class first and a full-rate op of another wave second, "
                                            "so at most 2 x min(B, (A+B)/2) / (A+B) of the ops can share a slot"}
        roof["executed"] = ex
    if stale:
        # no profile of THIS code object: its fields stay null rather than
        # borrowing another build's numbers
        roof["profile_stale"] = True
        roof["profile_missing"] = stale
    mix_w = workload_mix(len(cfg["msg"]), lo, hi)
    if mix_w and k_rate > 0:
        ipn_loop = mix_w[0] + mix_w[1]
        roof["work_bound"] = {"loop_valu_per_nonce": ipn_loop, "frac": ipn_loop * k_rate / VALU_PEAK_OPS,
                              "source": VARIANT_PROFILE,
                              "note": "per-nonce loop VALU of the variants this workload runs x this run's kernel "
                                      "rate / peak: a floor on the executed fraction; above 1 the line is refused"}
    if cfg["b_tail"] != 1:
        # the algorithmic count charges both tail blocks per nonce; the kernel
        # compresses the hi-digit block once per 10^k nonces and reads the
        # lo-only block's schedule from a table (MODE 5): the algorithmic
        # rate is not a utilisation, so it is not called a fraction here
        roof["alg_ops_over_peak"] = roof.pop("frac")
        roof.pop("frac_kind")
        roof["frac"] = (roof.get("executed") or {}).get("frac")
        roof["frac_basis"] = ("executed VALU lane-instructions (PMC) / peak: for this 2-block config the "
                              "algorithmic count overstates the work (block 0 once per 10^k nonces, block 1's "
                              "schedule tabulated), see alg_ops_over_peak")
        if "frac_rocprof" in roof:
            roof["alg_ops_over_peak_rocprof"] = roof.pop("frac_rocprof")
        if "frac_at_sustained_clock" in roof:
            roof["alg_ops_over_peak_at_sustained_clock"] = roof.pop("frac_at_sustained_clock")
    mix = mix_roofline()
    if mix and k_ms > 0:
        mix["peak_GH_s"] = mix["peak_GH_s_per_block"] / cfg["b_tail"]
        mix["speed_vs_unhoisted_mix"] = k_rate / 1e9 / mix["peak_GH_s"]
        mix["note"] = ("kernel rate / the rate the FULL algorithmic compression would reach with every "
                       "instruction at its own measured peak: a speed ratio, not a utilisation (the kernel "
                       "hoists per-thread rounds and schedule words, so it can exceed 1)")
        roof["unhoisted_mix"] = mix
    check_work_bound(roof)
    return roof


def scaling_expectation(config, n, codeobj=None):
    """What an N-GPU c4 run should reach if every GPU runs like the one this
    code object was profiled on: N x the one-GPU rate of the committed
    rocprofv3 c4 trace of THIS code object (2^38 / its average timed
    launch), divided by the slowest-over-mean shard time of N plan_shards
    shards, each timed alone on one GPU (tools/shard_balance.py, the newest
    profiles/*_shard_balance.jsonl).  Falls back to that file's own
    implied rate (its build's) when this code object has no c4 trace.  None
    for other configs or N without a balance measurement."""
    if config != "c4" or n < 2:
        return None
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_shard_balance.jsonl")), key=profile_tag_key)
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            rows = [json.loads(ln) for ln in f if ln.startswith("{")]
    except (OSError, ValueError):
        return None
    row = next((d for d in rows if d.get("n") == n and d.get("split") == "plan_shards"), None)
    if row is None:
        return None
    m = row["max_over_mean"]
    out = {"slowest_shard_over_mean": m, "shard_kernel_ms": row.get("kernel_ms"),
           "balance_source": os.path.relpath(files[-1], ROOT)}
    avg_ns, src = rocprof_row("c4", codeobj)
    if avg_ns:
        one = CONFIGS["c4"]["total"] / (avg_ns * 1e-9) / 1e9
        out.update(implied_GH_s=n * one / m, one_gpu_GH_s=one, one_gpu_source=src,
                   note="N x this code object's one-GPU c4 kernel rate (rocprofv3 trace) / the slowest "
                        "plan_shards shard over the mean; a shortfall against it is cross-GPU (see per_gpu)")
    else:
        out.update(implied_GH_s=row["implied_GH_s"], one_gpu_source=None,
                   note="2^38 / the slowest plan_shards shard timed alone on one GPU, on the build of "
                        "balance_source (no c4 trace of this code object is committed)")
    return out


def device_identity(index):
    """Ordinal, PCI bus id, UUID, arch and host of a device the library
    opened (p1hip_device_info), for the per-GPU records."""
    import socket

    import p1_amd

    info = p1_amd.device_info(index)
    return {"hostname": socket.gethostname(), "ordinal": info["ordinal"], "pci_bus_id": info["pci_bus_id"],
            "uuid": info["uuid"], "arch": info["arch"], "cu_count": info["cu_count"]}


class TopologyError(SystemExit):
    pass


def library_topology(mode, n_gpus, comms):
    """The `topology` block of a library-mode run (one process, p1hip_init(N))
    from what RCCL itself reports per device (p1_amd.comm_info:
    ncclCommCount / ncclCommUserRank).  For N > 1 every device must sit in an
    N-rank communicator and the ranks must be 0..N-1 once each, or the
    all-gather inside p1hip_scan does not span the N GPUs: TopologyError
    (bench.py exits 5 before timing anything).  N = 1 has no communicator
    (0 ranks)."""
    sizes = [int(c[0]) for c in comms]
    ranks = [int(c[1]) for c in comms]
    if len(comms) != n_gpus:
        raise TopologyError(f"bench.py: {len(comms)} devices open, --gpus {n_gpus}")
    if n_gpus > 1:
        if any(s != n_gpus for s in sizes) or sorted(ranks) != list(range(n_gpus)):
            raise TopologyError(f"bench.py: --gpus {n_gpus} but the library's RCCL communicators report sizes "
                                f"{sizes} and ranks {ranks}: the all-gather would not span {n_gpus} GPUs")
        backend, world, gather = "rccl (ncclCommInitAll in libp1hip)", n_gpus, n_gpus
    else:
        backend, world, gather = (None, 1, None) if sizes == [0] else ("rccl (forced, one rank)", sizes[0], sizes[0])
    return {"launch": mode, "backend": backend, "processes": 1, "world_size": world, "ranks_in_gather": gather,
            "rccl_ranks": sizes, "rccl_rank": ranks,
            "source": "p1hip_comm_info (ncclCommCount / ncclCommUserRank of each device's communicator)"}


class Progress:
    """A line on stderr at most every `every` seconds (rank 0 only): a c4
    run at N = 1 takes minutes before its one stdout line, and a silent
    process looks hung to a watchdog.  stdout stays the single JSON line."""

    def __init__(self, label, on=True, every=15.0):
        self.label, self.on, self.every = label, on, every
        self.last = time.perf_counter()

    def __call__(self, what, i, n):
        now = time.perf_counter()
        if self.on and (now - self.last >= self.every or i == n):
            print(f"bench.py: {self.label} {what} {i}/{n}", file=sys.stderr, flush=True)
            self.last = now


def timed_steps(step, steps, warmup, barrier, progress=None, probe=None):
    """W untimed steps, then K timed ones bracketed by barrier() (a
    torch.distributed barrier + device synchronise); library stats reset and
    HIP-event profiling on over exactly the timed steps.  With a ClockProbe,
    one clock stamp just before the opening barrier and one just after the
    closing one: the sustained shader clock of the timed steps (the stamps
    themselves are outside the timed region).  Returns (elapsed, step_ms,
    results, stats, clock)."""
    import p1_amd

    progress = progress or (lambda *a: None)
    for i in range(warmup):
        step()
        progress("warm-up step", i + 1, warmup)
    p1_amd.reset_stats()
    p1_amd.set_profiling(True)
    before = probe.stamp() if probe else None
    barrier()
    t0 = time.perf_counter()
    results, marks = [], [t0]
    for i in range(steps):
        results.append(step())  # synchronous: the (hash, nonce) result is on the host
        marks.append(time.perf_counter())
        progress("timed step", i + 1, steps)  # a few µs between steps, after the mark
    barrier()
    elapsed = time.perf_counter() - t0
    after = probe.stamp() if probe else None
    p1_amd.set_profiling(False)
    step_ms = sorted((b - a) * 1e3 for a, b in zip(marks, marks[1:]))
    clock = probe.clock(before, after) if probe else None
    if clock is not None:
        clock["timed_region_s"] = elapsed
    return elapsed, step_ms, results, p1_amd.get_stats(), clock


# by_config sub-results of the N = 1 line: (config, warmup, steps)
SUB_CONFIGS = [("c2", 2, 5), ("c3", 1, 3)]


def sub_result(name, warmup, steps, sync, codeobj=None, probe=None):
    """One other BASELINE config timed on the same device after the headline
    run: value, ms_per_step, the roofline fraction and the check against its
    independently pinned answer."""
    import p1_amd

    cfg = CONFIGS[name]
    total = job_total(cfg, 1)
    elapsed, step_ms, results, stats, clock = timed_steps(lambda: p1_amd.scan(cfg["msg"], 0, total - 1), steps,
                                                          warmup, sync, Progress(name), probe)
    pmc, pmc_src = pmc_summary(name, codeobj)
    roof = assemble_roofline(name, cfg, stats, steps, pmc, pmc_src, rocprof_row(name, codeobj), codeobj=codeobj,
                             clock=clock)
    known, src = known_answer(cfg, 1)
    res = results[-1]
    out = {"workload": cfg["desc"], "value": total * steps / elapsed / 1e9, "unit": "GH/s",
           "steps": steps, "warmup": warmup, "ms_per_step": elapsed * 1e3 / steps,
           "kernel_hashes_per_s_G": roof["kernel_hashes_per_s_G"], "avg_launch_ms": roof["avg_launch_ms"],
           "frac": roof["frac"], "result": list(res), "consistent": all(r == res for r in results),
           "matches_known": (tuple(res) == tuple(known)) if known else None, "known_source": src}
    for k in ("frac_rocprof", "alg_ops_over_peak", "alg_ops_over_peak_rocprof", "frac_basis", "rocprof_source",
              "effective_clock_GHz", "frac_at_sustained_clock", "profile_stale"):
        if k in roof:
            out[k] = roof[k]
    ex = roof.get("executed") or {}
    out["executed_frac"] = ex.get("frac")
    out["pmc_source"] = ex.get("source")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default=None,
                    help="default: c4 (configs[3], the fixed [0,2^38) job) at every N")
    ap.add_argument("--layout", default=None, metavar="L,START[,N]",
                    help="profile one tail layout instead of a BASELINE config (tools/sweep.py message of L bytes, "
                         "nonces [START, START+N), N default 2^32)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-small-request", action="store_true",
                    help="skip the configs[0]-sized latency probe (profiling runs: keeps every "
                         "k_scan launch in the rocprof summary a workload launch)")
    ap.add_argument("--no-by-config", action="store_true",
                    help="skip the c2/c3 sub-results of the N = 1 line (profiling runs)")
    ap.add_argument("--dist", action="store_true",
                    help="take the one-process-per-GPU torch.distributed path even when WORLD_SIZE is 1 "
                         "(rehearses the driver's N>1 launch, RCCL included, on one GPU)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torchrun path: nccl = RCCL over xGMI (production); gloo only to rehearse "
                         "several ranks on one GPU")
    args = ap.parse_args()

    # torch first: its wheel carries its own HIP runtime, and libp1hip.so must
    # bind to that already-loaded copy.  Loaded the other way round, the
    # process holds two HIP runtimes and whichever initialises second sees no
    # device (r04a: "No HIP GPUs are available" / p1hip rc -1).
    import torch

    import p1_amd
    from p1_amd.build import ensure_built

    ensure_built()
    # production settings only: refuse before any device is touched
    knobs = p1_amd.test_knobs()
    if knobs:
        print(f"bench.py: refusing to time with library test knobs in force: {knobs} "
              f"(unset P1HIP_TEST_KNOBS)", file=sys.stderr)
        sys.exit(4)

    visible = torch.cuda.device_count()
    try:
        run = resolve_run(args.gpus, args.config, os.environ,
                          visible if args.dist_backend == "nccl" else max(visible, args.gpus), args.dist)
    except UsageError as e:
        print(str(e), file=sys.stderr)
        sys.exit(2)
    if args.layout:
        try:
            cfg = layout_config(args.layout)
        except UsageError as e:
            print(str(e), file=sys.stderr)
            sys.exit(2)
        run["config"] = "L%dd%d" % tuple(cfg["layout"])
    else:
        cfg = CONFIGS[run["config"]]
    mode, n_gpus, rank, world = run["mode"], run["n"], run["rank"], run["world"]

    import torch.distributed as dist

    from p1_amd.dist import distributed_scan

    msg = cfg["msg"]
    total = job_total(cfg, n_gpus)
    base = cfg.get("lo", 0)  # first nonce of the job
    t_init = time.perf_counter()  # device init, module load, communicators: reported, not timed
    if mode == "torchrun":
        gpu = run["local_rank"] % visible if args.dist_backend == "gloo" else run["local_rank"]
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
        p1_amd.init_devices([gpu])
        devices = [gpu]
        coll_dev = torch.device("cuda", gpu) if args.dist_backend == "nccl" else torch.device("cpu")
        sync_devs = [gpu]
    else:
        got = p1_amd.init(n_gpus)
        if got != n_gpus:
            print(f"bench.py: library opened {got} devices, asked for {n_gpus}", file=sys.stderr)
            sys.exit(2)
        devices = list(range(n_gpus))
        sync_devs = devices
        comms = [p1_amd.comm_info(i) for i in range(got)]
        try:
            lib_topology = library_topology(mode, n_gpus, comms)
        except TopologyError as e:
            print(str(e), file=sys.stderr)
            sys.exit(5)
    init_ms = (time.perf_counter() - t_init) * 1e3
    codeobj = p1_amd.codeobj_sha256()
    # HIP ordinals of the devices this process scans on, for the clock probe
    ordinals = [gpu] if mode == "torchrun" else [p1_amd.device_info(i)["ordinal"] for i in devices]
    probe = ClockProbe(ordinals)

    timing = {}  # torchrun: this rank's scan / all-gather time of the timed steps

    def step():
        if mode == "torchrun":
            return distributed_scan(msg, base, base + total - 1, p1_amd.scan, device=coll_dev, shard_fn=p1_amd.plan_shards,
                                    timing=timing)
        return p1_amd.scan(msg, base, base + total - 1)  # library: shards + RCCL all-gather inside

    def barrier():
        if mode == "torchrun":
            dist.barrier()
        for d in sync_devs:
            torch.cuda.synchronize(d)

    progress = Progress(run["config"], on=(rank == 0))
    for i in range(args.warmup):
        step()
        progress("warm-up step", i + 1, args.warmup)
    timing.clear()
    elapsed, step_ms, results, stats, clock = timed_steps(step, args.steps, 0, barrier, progress, probe)

    if mode == "torchrun":
        from p1_amd.dist import gather_rank_identity, gather_rank_stats

        shard = timing.get("shard")
        units = gather_rank_stats({
            "shard_lo": shard[0] if shard else 1, "shard_hi": shard[1] if shard else 0,
            "nonces": stats["scan_nonces"], "launches": stats["scan_launches"], "alg_ops": stats["scan_alg_ops"],
            "kernel_ms": stats["scan_kernel_ms"], "scan_ms": timing.get("scan_s", 0.0) * 1e3,
            "gather_ms": timing.get("gather_s", 0.0) * 1e3, "elapsed_ms": elapsed * 1e3,
            "step_ms_median": statistics.median(step_ms) if step_ms else 0.0}, device=coll_dev)
        idents = gather_rank_identity(dict(device_identity(0), rank=rank), device=coll_dev)
        for u, ident in zip(units, idents):
            u["identity"] = ident
        elapsed = max(u["elapsed_ms"] for u in units) / 1e3  # max over ranks
        topology = {"launch": "torchrun", "backend": dist.get_backend(), "world_size": dist.get_world_size(),
                    "ranks_in_gather": len(idents)}
    else:
        units = []
        for i in range(len(devices)):
            ds = p1_amd.get_device_stats(i)
            units.append({"device": i, "ordinal": ds["ordinal"], "identity": device_identity(i),
                          "shard_lo": ds["shard_first"], "shard_hi": ds["shard_last"] if ds["active"] else 0,
                          "nonces": ds["scan_nonces"], "launches": ds["scan_launches"],
                          "alg_ops": ds["scan_alg_ops"], "kernel_ms": ds["scan_kernel_ms"],
                          "scan_ms": ds["phase1_ms"], "gather_ms": ds["gather_ms"],
                          "rccl_ranks": comms[i][0], "rccl_rank": comms[i][1]})
            if not ds["active"]:
                units[-1]["shard_lo"] = 1
        topology = lib_topology
    gpus_seen = {(u["identity"]["hostname"], u["identity"]["pci_bus_id"], u["identity"]["uuid"]) for u in units}
    topology["distinct_gpus"] = len(gpus_seen)
    topology["hosts"] = sorted({h for h, _, _ in gpus_seen})

    result = results[-1]
    consistent = all(r == result for r in results)
    roof_failed = []
    known, known_src = known_answer(cfg, n_gpus)

    if rank == 0:
        hashes = total * args.steps
        value = hashes / elapsed / 1e9
        ms_per_step = elapsed * 1e3 / args.steps
        pmc, pmc_src = pmc_summary(run["config"], codeobj)
        try:
            roofline = assemble_roofline(run["config"], cfg, stats, args.steps, pmc, pmc_src,
                                         rocprof_row(run["config"], codeobj), single_gpu=(n_gpus == 1),
                                         codeobj=codeobj, clock=clock)
        except RooflineError as e:
            # the line is still printed (minutes of timing are not thrown
            # away), the error named in it, and the exit status says so
            roofline = {"error": str(e), "bound": "valu-int32", "frac": None}
            roof_failed.append(str(e))
        parallelism = {"single": "1 GPU",
                       "library": f"cost-balanced contiguous range-shard x{n_gpus} (p1hip_plan_shards), one process (p1hip_init({n_gpus}): thread per device, "
                                  f"ncclCommInitAll + ncclAllGather of 16-B partials)",
                       "torchrun": f"cost-balanced contiguous range-shard x{n_gpus} (p1hip_plan_shards), "
                                   "one process per GPU + "
                                   + ("RCCL all-gather (torch.distributed nccl)" if args.dist_backend == "nccl"
                                      else "gloo all-gather (rehearsal)")}[mode]
        line = {
            "metric": "SHA-256 nonce-hashes/sec (GH/s)",
            "value": value,
            "unit": "GH/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            # SURVEY.md 8(d) timing: per-step wall times (first enqueue to the
            # host min) of this rank, median of the K steps; one-time setup
            # (devices, code object, communicators) is outside the timed region
            "step_ms": {"median": statistics.median(step_ms), "min": step_ms[0], "max": step_ms[-1],
                        "n": len(step_ms), "rank": rank} if step_ms else None,
            "init_ms": init_ms,
            "higher_is_better": True,
            "scaling": "strong" if "total" in cfg else "weak",
            "vs_baseline": value * 1e9 / PUBLISHED_HASHES_PER_S,
            "vs_baseline_basis": "value / the reference's published bitcoin.Hash rate, 'around 10,000 per "
                                 "second' (p1.pdf 4.1, BASELINE.md 1)",
            "dtype": "u32",
            "data": "synthetic",
            "config": {
                "workload": cfg["desc"],
                "config": run["config"],
                "msg_len": len(msg),
                "nonces_per_gpu": total // n_gpus,
                "job_range": [base, base + total - 1],
                "parallelism": parallelism,
                "launch": mode,
                "devices": devices if mode != "torchrun" else f"one per rank, {world} ranks",
            },
            "test_knobs": knobs,
            "library": {"path": os.path.relpath(p1_amd.lib_path(), ROOT), "version": p1_amd.version(),
                        "codeobj_sha256": codeobj},
            "topology": topology,
            "scaling_expectation": scaling_expectation(run["config"], n_gpus, codeobj),
            "roofline": roofline,
            "per_gpu": scaling_report(units, args.steps, ms_per_step),
            "result": {"hash": result[0], "nonce": result[1], "consistent": consistent,
                       "matches_known": (tuple(result) == tuple(known)) if known else None,
                       "known": list(known) if known else None, "known_source": known_src},
        }
        if "layout" in cfg:
            line["config"].update(layout=cfg["layout"], variant=cfg["variant"], b_tail=cfg["b_tail"])
        if n_gpus == 1 and mode != "torchrun" and not args.no_by_config and "layout" not in cfg:
            # the other BASELINE configs on the same GPU, after the timed
            # headline run (never inside it)
            line["by_config"] = {run["config"]: {"value": value, "ms_per_step": ms_per_step,
                                                 "frac": roofline.get("frac"),
                                                 "effective_clock_GHz": roofline.get("effective_clock_GHz"),
                                                 "matches_known": line["result"]["matches_known"],
                                                 "headline": True}}
            for name, w, k in SUB_CONFIGS:
                if name != run["config"]:
                    try:
                        line["by_config"][name] = sub_result(name, w, k, barrier, codeobj, probe)
                    except RooflineError as e:
                        line["by_config"][name] = {"error": str(e)}
                        roof_failed.append(f"{name}: {e}")
        # configs[0]'s request (client 'bradfitz' maxNonce 9999) as one
        # drop-in call: per-request latency of p1hip_scan on a small job
        lat = []
        for _ in range(0 if args.no_small_request else 20):
            t0 = time.perf_counter()
            small = p1_amd.scan(b"bradfitz", 0, 9999)
            lat.append(time.perf_counter() - t0)
        lat.sort()
        if lat:
            line["small_request"] = {"request": "bradfitz [0, 9999] (configs[0])", "result": list(small),
                                     "matches_known": tuple(small) == (1419516646206828, 9898),
                                     "median_latency_us": lat[len(lat) // 2] * 1e6}
        if n_gpus == 1 and not args.no_cpu:
            print("bench.py: cpu_baseline", file=sys.stderr, flush=True)
            line["cpu_baseline"] = cpu_baseline(msg, 1 << 31, args.cpu_seconds)
        print(json.dumps(line), flush=True)
        wrong = [k for k, v in line.get("by_config", {}).items() if v.get("matches_known") is False]
    else:
        wrong = []

    if mode == "torchrun":
        dist.destroy_process_group()
    p1_amd.shutdown()
    if (known and tuple(result) != tuple(known)) or wrong:
        sys.exit(3)  # a wrong answer is not a benchmark result
    if roof_failed:
        print(f"bench.py: roofline refused: {roof_failed}", file=sys.stderr)
        sys.exit(6)


if __name__ == "__main__":
    main()
