"""Throughput of p1hip_scan across tail layouts (GPU box).

For message lengths 0..127 (every (L+1) mod 64 phase, 1- and 2-block tails,
PRE/TRAIL/straddle variants) scans SWEEP_NONCES nonces (default 2^32, the
configs[1] size) starting at 10^9 (d = 10) and at 10^15 (d = 16).  Each case
is warmed up with the same scan first; the rate is taken from the k_scan
HIP-event time (library profiling, as bench.py does) and from the host wall
time of p1hip_scan.  The reported nonce must re-hash to the reported hash
(oracle).  Prints one JSON line per case and a summary line.

Per case: the fast variant (FV, MODE, TRAIL) the planner picks, the algorithmic
roofline fraction (1384 x B_tail ops per nonce at the kernel rate over
78.64 TOP/s, the bench.py accounting).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402  (checker only)
import p1_amd  # noqa: E402
from bench import fast_variant  # noqa: E402

PEAK = 256 * 4 * 32 * 2.4e9


def variant(L, d):
    """(FV, MODE, TRAIL) of the fast path for message length L, d digits."""
    return fast_variant(L, d)


def main():
    n = int(os.environ.get("SWEEP_NONCES", 1 << 32))
    lengths = [int(x) for x in os.environ.get("SWEEP_LENGTHS", "").split(",") if x] or list(range(0, 128))
    starts = [int(x) for x in os.environ.get("SWEEP_STARTS", "").split(",") if x] or [10**9, 10**15]
    p1_amd.init_devices([0])
    rows = []
    for L in lengths:
        m = bytes((33 + (i * 7) % 90) for i in range(L))
        for start in starts:
            p1_amd.scan(m, start, start + n - 1)  # warm (clocks, caches, allocations)
            p1_amd.reset_stats()
            p1_amd.set_profiling(True)
            t0 = time.perf_counter()
            h, nn = p1_amd.scan(m, start, start + n - 1)
            dt = time.perf_counter() - t0
            p1_amd.set_profiling(False)
            st = p1_amd.get_stats()
            ok = oracle.hash(m, nn) == h
            d = len(str(start))
            r = (L + 1) % 64
            btail = 1 if r + d + 9 <= 64 else 2
            kgh = st["scan_nonces"] / (st["scan_kernel_ms"] * 1e-3) / 1e9
            row = {"L": L, "d": d, "B_tail": btail, "variant": variant(L, d), "GH_s": kgh,
                   "wall_GH_s": n / dt / 1e9, "frac": kgh * 1e9 * 1384 * btail / PEAK, "rehash_ok": ok}
            rows.append(row)
            print(json.dumps(row), flush=True)
    by = {}
    for r in rows:
        by.setdefault(r["B_tail"], []).append(r)
    print(json.dumps({"summary": {f"B_tail={k}": {"min_GH_s": min(x["GH_s"] for x in v),
                                                   "max_GH_s": max(x["GH_s"] for x in v),
                                                   "mean_GH_s": sum(x["GH_s"] for x in v) / len(v),
                                                   "min_frac": min(x["frac"] for x in v),
                                                   "worst": min(v, key=lambda x: x["frac"])}
                                  for k, v in by.items()},
                      "nonces_per_case": n, "all_rehash_ok": all(r["rehash_ok"] for r in rows)}))


if __name__ == "__main__":
    main()
