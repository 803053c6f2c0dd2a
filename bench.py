#!/usr/bin/env python3
"""bench.py -- nonce-scan throughput of libp1hip.so on MI355X.

Metric (BASELINE.json): SHA-256 nonce-hashes/s (GH/s) at 1/2/4/8 MI355X and
the fraction of the integer-VALU roofline.

Workload (BASELINE.json configs[1], "c2"): msg = "bradfitz" (8 bytes), the
nonce range [0, 2^32) per GPU -- one SHA-256 compression per nonce.  A step
is one full scan of that range (the drop-in for miner.go:56-63) ending with
the (hash, nonce) result on the host.  With N GPUs (torchrun, one process per
GPU) the job range is [0, N*2^32), sharded contiguously (weak scaling); the
16-byte per-rank results are all-gathered over RCCL (torch.distributed
"nccl") and reduced with the lexicographic (hash, nonce) min.  `--config c3`
selects configs[2] (120-byte msg, 2^34 nonces per GPU, 2 tail blocks);
`--config c4` selects configs[3] (the fixed [0, 2^38) job split over the GPUs,
strong scaling).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# int32 VALU peak of one MI355X: 256 CUs x 4 SIMD x 32 lanes (wave64 VALU op
# issues in 2 cycles on CDNA4's SIMD-32, MI355X_MICROARCH.md "Execution model")
# x 2.4 GHz max clock.  tools/valu_peak measures the per-instruction rates
# (profiles/r01_valu_peak.jsonl).
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9
# SURVEY.md 8(d)'s peak assumed 64 int32 lane-ops/clk/CU (39.32 T/s); the
# measured rates are 2x that for bitop3/add/xor and equal to it for
# alignbit/add3 (profiles/r01_valu_peak.jsonl), so it is reported beside.
SURVEY_PEAK_OPS = 39.32e12
ALG_OPS_PER_COMPRESSION = 1384  # 64 rounds x 14 + 48 schedule words x 10 + 8

CONFIGS = {
    "c2": {"msg": b"bradfitz", "per_gpu": 1 << 32, "b_tail": 1,
           "desc": "configs[1]: 8-byte msg 'bradfitz', nonces [0,2^32) per GPU, 1 SHA-256 block/nonce",
           "known": {1: (5256245051, 1626825724)}},
    "c3": {"msg": b"cmu440-p1-" * 12, "per_gpu": 1 << 34, "b_tail": 2,
           "desc": "configs[2]: 120-byte msg, host midstate, nonces [0,2^34) per GPU, 2 tail blocks/nonce",
           "known": {}},
    # configs[3]: the fixed 2^38 job split over however many GPUs run (strong scaling)
    "c4": {"msg": b"bradfitz", "total": 1 << 38, "b_tail": 1,
           "desc": "configs[3]: 8-byte msg 'bradfitz', nonces [0,2^38) split contiguously over the GPUs",
           "known": {}},
}


# The algorithmic SHA-256 compression (SURVEY.md 8(d)'s 1384 ops) by
# instruction class: 64 rounds x (6 rotr, 4 bitop3, 3 add3, 1 add) +
# 48 schedule words x (4 rotr, 2 shr, 2 bitop3, 1 add3, 1 add) + 8 adds.
ALG_MIX = {"v_alignbit_b32": 576, "v_bitop3_b32": 352, "v_add3_u32": 240, "v_add_u32": 120,
           "v_lshrrev_b32": 96}
VALU_PEAK_PROFILE = "profiles/r01_valu_peak.jsonl"


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


def pmc_traffic():
    """HBM bytes per k_scan launch from the newest committed rocprofv3 PMC
    summary (profiles/*_pmc_summary.json, FETCH_SIZE + WRITE_SIZE of the c2
    workload, collected in separate --pmc passes by tools/gpu_round.sh)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def cpu_baseline(msg, start, target_s):
    """Oracle restatement (format + full SHA-256 per nonce, the reference's
    per-nonce work) on the host cores, bounded sample."""
    import oracle

    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or min(16, os.cpu_count() or 1)
    cal = 1 << 18
    t0 = time.perf_counter()
    oracle.scan(msg, start, start + cal * threads - 1, threads=threads)
    rate = cal * threads / (time.perf_counter() - t0)
    n = max(int(rate * target_s), cal * threads)
    t0 = time.perf_counter()
    oracle.scan(msg, start, start + n - 1, threads=threads)
    dt = time.perf_counter() - t0
    return {
        "value": n / dt / 1e9,
        "unit": "GH/s",
        "cores": threads,
        "kind": "port",
        "sample": f"oracle/p1_oracle.c (C restatement of hash.go:13-17 + miner.go:56-63, sprintf-equivalent "
                  f"formatting + full SHA-256 per nonce), {threads} threads, nonces [{start}, {start + n - 1}] "
                  f"({n} nonces, {dt:.1f} s) of the same message",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-small-request", action="store_true",
                    help="skip the configs[0]-sized latency probe (profiling runs: keeps every "
                         "k_scan launch in the rocprof summary a workload launch)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo only to rehearse "
                         "several ranks on one GPU")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    cfg = CONFIGS[args.config]

    import torch
    import torch.distributed as dist

    import p1_amd
    from p1_amd.build import ensure_built
    from p1_amd.dist import distributed_scan

    ensure_built()

    ngpu = torch.cuda.device_count()
    gpu = local % ngpu if args.dist_backend == "gloo" else local  # gloo rehearsal may share a GPU
    if world > 1:
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    p1_amd.init_devices([gpu])

    msg = cfg["msg"]
    total = cfg["total"] if "total" in cfg else cfg["per_gpu"] * world
    shard = p1_amd.shard_range(0, total - 1, rank, world)
    dev = torch.device("cuda", gpu)
    coll_dev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    def step():
        if world == 1:
            return p1_amd.scan(msg, shard[0], shard[1])
        return distributed_scan(msg, 0, total - 1, p1_amd.scan, device=coll_dev)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    p1_amd.reset_stats()
    p1_amd.set_profiling(True)
    barrier()
    t0 = time.perf_counter()
    results = [step() for _ in range(args.steps)]
    barrier()
    elapsed = time.perf_counter() - t0
    p1_amd.set_profiling(False)
    stats = p1_amd.get_stats()

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    result = results[-1]
    consistent = all(r == result for r in results)
    known = cfg["known"].get(world)

    if rank == 0:
        hashes = total * args.steps
        value = hashes / elapsed / 1e9
        ms_per_step = elapsed * 1e3 / args.steps
        traffic, traffic_src = pmc_traffic() if args.config == "c2" else (None, None)
        k_ms = stats["scan_kernel_ms"]
        k_n = stats["scan_launches"]
        achieved = stats["scan_alg_ops"] / (k_ms * 1e-3) if k_ms > 0 else 0.0
        roofline = {
            "bound": "valu-int32",
            "achieved": achieved / 1e12,
            "peak": VALU_PEAK_OPS / 1e12,
            "unit": "TOP/s",
            "frac": achieved / VALU_PEAK_OPS,
            "traffic": traffic,
            "traffic_unit": "bytes/launch (PMC FETCH_SIZE+WRITE_SIZE)",
            "traffic_source": traffic_src,
            "kernel": "k_scan (one launch per scan covers every decade; algorithmic ops = 1384 x B_tail per nonce)",
            "alg_ops_per_nonce": ALG_OPS_PER_COMPRESSION * cfg["b_tail"],
            "avg_launch_ms": k_ms / k_n if k_n else None,
            "launches_per_step": k_n / args.steps,
            "kernel_hashes_per_s_G": stats["scan_nonces"] / (k_ms * 1e-3) / 1e9 if k_ms > 0 else None,
            "frac_vs_survey_peak": achieved / SURVEY_PEAK_OPS,
            "fast_nonce_share": stats["fast_nonces"] / max(1, stats["fast_nonces"] + stats["generic_nonces"]),
        }
        mix = mix_roofline()
        if mix and k_ms > 0:
            khs = stats["scan_nonces"] / (k_ms * 1e-3) / 1e9
            mix["peak_GH_s"] = mix["peak_GH_s_per_block"] / cfg["b_tail"]
            mix["frac"] = khs / mix["peak_GH_s"]
            roofline["mix_roofline"] = mix
        line = {
            "metric": "SHA-256 nonce-hashes/sec (GH/s)",
            "value": value,
            "unit": "GH/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if "total" in cfg else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {
                "workload": cfg["desc"],
                "msg_len": len(msg),
                "nonces_per_gpu": total // world,
                "job_range": [0, total - 1],
                "parallelism": f"range-shard x{world}" + (
                    (" + RCCL all-gather" if args.dist_backend == "nccl" else " + gloo all-gather (rehearsal)")
                    if world > 1 else ""),
            },
            "roofline": roofline,
            "result": {"hash": result[0], "nonce": result[1], "consistent": consistent,
                       "matches_known": (tuple(result) == known) if known else None},
        }
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
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(msg, 1 << 31, args.cpu_seconds)
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.destroy_process_group()
    p1_amd.shutdown()


if __name__ == "__main__":
    main()
