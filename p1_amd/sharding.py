"""Contiguous nonce-range sharding and the cross-shard min, for the
one-process-per-GPU path (bench.py under torchrun).

Reference semantics: miner.go:56-63 -- inclusive range, strict '<' so the
lowest nonce wins ties, identity (MaxUint64, 0).  A contiguous split plus a
lexicographic (hash, nonce) min over shard results reproduces the serial
first-minimum exactly; see SURVEY.md 8(e).
"""
U64_MAX = (1 << 64) - 1


def shard_range(lower, upper, rank, world):
    """Return the inclusive [lo, hi] of shard `rank`, or None if it is empty.

    Shard sizes differ by at most one and cover [lower, upper] in order."""
    if lower > upper:
        return None
    count = upper - lower + 1
    per, extra = divmod(count, world)
    size = per + (1 if rank < extra else 0)
    if size == 0:
        return None
    lo = lower + rank * per + min(rank, extra)
    return lo, lo + size - 1


def combine_keys(keys):
    """Lexicographic min of per-shard (hash, nonce) results.

    Each input is a shard's (hash, nonce) exactly as p1hip_scan returns it
    (so an all-UINT64_MAX shard reads (U64_MAX, 0)); the result follows the
    same rule: nonce 0 when the minimum hash is U64_MAX."""
    best = None
    for h, n in keys:
        if h == U64_MAX:
            continue
        if best is None or (h, n) < best:
            best = (h, n)
    return best if best is not None else (U64_MAX, 0)
