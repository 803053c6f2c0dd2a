"""Multi-GPU shard balance, measured on one GPU.

An N-GPU scan of configs[3] ([0, 2^38) for "bradfitz") ends when its
slowest shard ends.  This tool scans each of the N shards in turn on GPU 0,
times its k_scan launch with HIP events (p1hip stats, profiling on), and
reports for the equal-count split (sharding.shard_range) and for the
library's cost-balanced split (p1hip_plan_shards): the per-shard kernel
times, max/mean (1.0 = every rank finishes together) and the N-GPU rate the
slowest shard implies (2^38 / max).  One JSON line per (N, split).

usage: python tools/shard_balance.py [N ...]   (default 2 4 8)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import p1_amd  # noqa: E402
from p1_amd.build import ensure_built  # noqa: E402

MSG = b"bradfitz"
TOTAL = 1 << 38


def shard_ms(lo, hi):
    p1_amd.reset_stats()
    got = p1_amd.scan(MSG, lo, hi)
    return p1_amd.get_stats()["scan_kernel_ms"], got


def main():
    ensure_built()
    ns = [int(x) for x in sys.argv[1:]] or [2, 4, 8]
    p1_amd.init_devices([0])
    p1_amd.set_profiling(True)
    shard_ms(0, (1 << 32) - 1)  # warm-up
    for n in ns:
        splits = {"equal": [p1_amd.shard_range(0, TOTAL - 1, r, n) for r in range(n)],
                  "plan_shards": p1_amd.plan_shards(MSG, 0, TOTAL - 1, n)}
        for name, shards in splits.items():
            times, keys = [], []
            for s in shards:
                ms, key = shard_ms(*s)
                times.append(ms)
                keys.append(key)
            mx, mean = max(times), sum(times) / len(times)
            print(json.dumps({"n": n, "split": name, "shards": shards, "kernel_ms": times,
                              "max_over_mean": mx / mean, "implied_GH_s": TOTAL / (mx * 1e-3) / 1e9,
                              "result": list(min(keys)), "codeobj_sha256": p1_amd.codeobj_sha256()}), flush=True)


if __name__ == "__main__":
    main()
