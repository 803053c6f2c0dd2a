"""Throughput of p1hip_scan across tail layouts (GPU box).

For message lengths 0..127 (every (L+1) mod 64 phase, 1- and 2-block tails,
PRE/TRAIL/straddle variants) scans 2^30 nonces starting at 10^9 (d = 10) and
at 10^15 (d = 16), checks the reported nonce re-hashes to the reported hash
(oracle), and prints one JSON line per case plus a summary line.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402  (checker only)
import p1_amd  # noqa: E402


def main():
    n = int(os.environ.get("SWEEP_NONCES", 1 << 30))
    lengths = [int(x) for x in os.environ.get("SWEEP_LENGTHS", "").split(",") if x] or list(range(0, 128))
    p1_amd.init_devices([0])
    rows = []
    for L in lengths:
        m = bytes((33 + (i * 7) % 90) for i in range(L))
        for start in (10**9, 10**15):
            p1_amd.scan(m, start, start + (1 << 20))  # warm
            t0 = time.perf_counter()
            h, nn = p1_amd.scan(m, start, start + n - 1)
            dt = time.perf_counter() - t0
            ok = oracle.hash(m, nn) == h
            d = len(str(start))
            r = (L + 1) % 64
            btail = 1 if r + d + 9 <= 64 else 2
            row = {"L": L, "d": d, "B_tail": btail, "GH_s": n / dt / 1e9, "rehash_ok": ok}
            rows.append(row)
            print(json.dumps(row), flush=True)
    by = {}
    for r in rows:
        by.setdefault(r["B_tail"], []).append(r["GH_s"])
    print(json.dumps({"summary": {f"B_tail={k}": {"min": min(v), "max": max(v), "mean": sum(v) / len(v)}
                                  for k, v in by.items()},
                      "all_rehash_ok": all(r["rehash_ok"] for r in rows)}))


if __name__ == "__main__":
    main()
