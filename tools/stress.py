"""Randomized parity stress of p1hip_scan (GPU box; test tool, not product).

Draws random requests -- message lengths 0..200 (every tail layout, MODE 5
included), ranges from 1 nonce to 10^9 nonces anywhere in the u64 range --
and checks each against the CPU oracle: bit-exact for ranges the oracle
finishes quickly (<= 2*10^6 nonces), and for larger ones by the size-free
properties (the nonce lies in the range and re-hashes to the hash; the
result equals the min of the two halves scanned separately).  Runs with the
production settings (one-launch small path, MODE 5 tables, default occupancy
floor).  Prints one JSON summary line.

usage: [STRESS_MAXLEN=n] python tools/stress.py [seconds] [seed]
(the fast-variant run forces k = 3 on small ranges with the test knobs
P1HIP_TEST_KNOBS=1 P1HIP_MIN_FAST_THREADS=1 P1HIP_SMALL_MAX_NONCES=0; the
summary line records the knobs in force)
"""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402  (checker only)
import p1_amd  # noqa: E402

U64_MAX = (1 << 64) - 1


MAX_LEN = int(os.environ.get("STRESS_MAXLEN", "200"))  # message lengths 0..MAX_LEN


def draw(rnd):
    L = rnd.randrange(0, MAX_LEN + 1)
    m = bytes(rnd.randrange(32, 127) for _ in range(L))
    size = int(10 ** rnd.uniform(0, 9))
    d = rnd.randrange(1, 21)
    base = 0 if d == 1 else 10 ** (d - 1)
    lo = min(base + int(rnd.random() * 10 ** (d - 1)) - rnd.randrange(0, 3) * size // 2, U64_MAX)
    lo = max(lo, 0)
    hi = min(lo + size - 1, U64_MAX)
    return m, lo, hi


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 440
    rnd = random.Random(seed)
    p1_amd.init_devices([0])
    oracle.load()
    t_end = time.time() + secs
    n_exact = n_prop = 0
    nonces = 0
    fails = []
    t_report = time.time() + 60
    while time.time() < t_end:
        if time.time() > t_report:  # progress for long runs (a silent GPU command looks hung)
            print(f"stress: {n_exact} exact, {n_prop} property, {len(fails)} failures so far", file=sys.stderr,
                  flush=True)
            t_report += 60
        m, lo, hi = draw(rnd)
        got = p1_amd.scan(m, lo, hi)
        nonces += hi - lo + 1
        if hi - lo < 2 * 10**6:
            want = oracle.scan(m, lo, hi, threads=16)
            n_exact += 1
            if got != want:
                fails.append({"msg_hex": m.hex(), "lower": lo, "upper": hi, "got": got, "want": want})
        else:
            n_prop += 1
            h, n = got
            mid = lo + (hi - lo) // 3
            ok = lo <= n <= hi and oracle.hash(m, n) == h
            ok = ok and min(p1_amd.scan(m, lo, mid), p1_amd.scan(m, mid + 1, hi)) == got
            if not ok:
                fails.append({"msg_hex": m.hex(), "lower": lo, "upper": hi, "got": got})
    print(json.dumps({"seed": seed, "seconds": secs, "requests_exact": n_exact, "requests_property": n_prop,
                      "nonces_scanned": nonces, "failures": fails[:20], "n_failures": len(fails),
                      "test_knobs": p1_amd.test_knobs(), "library": p1_amd.version()}), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
