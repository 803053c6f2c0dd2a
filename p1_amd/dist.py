"""One-process-per-GPU scan: contiguous shard per rank, 16-byte per-rank
results all-gathered over torch.distributed (backend "nccl" = RCCL over
xGMI on MI355X; "gloo" in the CPU tests), lexicographic (hash, nonce) min.

This is the only collective on the path: the reference has
no exchange step besides the final min of miner.go:56-63.
"""
import json
import time

import torch
import torch.distributed as dist

from .sharding import combine_keys, shard_range


def _to_i64(v):
    return v - (1 << 64) if v >= (1 << 63) else v


def _to_u64(v):
    return v + (1 << 64) if v < 0 else v


def distributed_scan(msg, lower, upper, scan_fn, device=None, group=None, shard_fn=None, timing=None):
    """Scan [lower, upper] with every rank of `group` taking one contiguous
    shard through scan_fn(msg, lo, hi) -> (hash, nonce); returns the global
    result on every rank.

    shard_fn(msg, lower, upper, world) -> [(lo, hi) | None] * world picks the
    shards (default: equal nonce counts, sharding.shard_range); the GPU path
    passes p1_amd.plan_shards, the library's cost-balanced contiguous split.
    Every rank must use the same shard_fn.  `timing` (a dict), when given,
    accumulates this rank's "scan_s" and "gather_s" (the all-gather and the
    host min, device synchronised) and records its last "shard"."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if shard_fn is None:
        s = shard_range(lower, upper, rank, world)
    else:
        s = shard_fn(msg, lower, upper, world)[rank]
    t0 = time.perf_counter()
    key = scan_fn(msg, s[0], s[1]) if s is not None else (2**64 - 1, 0)
    t1 = time.perf_counter()
    t = torch.tensor([_to_i64(key[0]), _to_i64(key[1])], dtype=torch.int64, device=device)
    out = torch.empty(2 * world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, t, group=group)
    v = [_to_u64(x) for x in out.tolist()]  # .tolist() waits for the collective
    res = combine_keys(list(zip(v[0::2], v[1::2])))
    if timing is not None:
        timing["scan_s"] = timing.get("scan_s", 0.0) + (t1 - t0)
        timing["gather_s"] = timing.get("gather_s", 0.0) + (time.perf_counter() - t1)
        timing["steps"] = timing.get("steps", 0) + 1
        timing["shard"] = s
    return res


# Per-rank accounting of a timed run, gathered so rank 0 can explain the
# scaling it reports (which shard each rank scanned, its kernel time, its
# collective time).  Integers travel as int64 (u64 two's complement), times
# as float64.
RANK_INT_FIELDS = ("shard_lo", "shard_hi", "nonces", "launches", "alg_ops")
RANK_FLOAT_FIELDS = ("kernel_ms", "scan_ms", "gather_ms", "elapsed_ms", "step_ms_median")


def gather_rank_stats(stats, device=None, group=None):
    """All-gather one dict per rank (keys RANK_INT_FIELDS + RANK_FLOAT_FIELDS);
    returns the list of every rank's dict, in rank order, on every rank."""
    world = dist.get_world_size(group)
    ti = torch.tensor([_to_i64(int(stats[k])) for k in RANK_INT_FIELDS], dtype=torch.int64, device=device)
    tf = torch.tensor([float(stats[k]) for k in RANK_FLOAT_FIELDS], dtype=torch.float64, device=device)
    oi = torch.empty(world * len(RANK_INT_FIELDS), dtype=torch.int64, device=device)
    of = torch.empty(world * len(RANK_FLOAT_FIELDS), dtype=torch.float64, device=device)
    dist.all_gather_into_tensor(oi, ti, group=group)
    dist.all_gather_into_tensor(of, tf, group=group)
    vi, vf = oi.tolist(), of.tolist()
    out = []
    ni, nf = len(RANK_INT_FIELDS), len(RANK_FLOAT_FIELDS)
    for r in range(world):
        d = {"rank": r}
        d.update({k: _to_u64(vi[r * ni + j]) for j, k in enumerate(RANK_INT_FIELDS)})
        d.update({k: vf[r * nf + j] for j, k in enumerate(RANK_FLOAT_FIELDS)})
        out.append(d)
    return out


IDENTITY_BYTES = 512


def gather_rank_identity(ident, device=None, group=None):
    """All-gather one small JSON-able dict per rank (host name, device
    ordinal, PCI bus id, UUID ...) as a fixed-size byte record over the same
    process group, so rank 0 can show which physical GPU each rank ran on.
    Returns the list of dicts in rank order."""
    world = dist.get_world_size(group)
    raw = json.dumps(ident, sort_keys=True).encode()
    if len(raw) > IDENTITY_BYTES:
        raise ValueError(f"identity record of {len(raw)} bytes > {IDENTITY_BYTES}")
    buf = torch.zeros(IDENTITY_BYTES, dtype=torch.uint8)
    buf[:len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    t = buf.to(device) if device is not None else buf
    out = torch.empty(world * IDENTITY_BYTES, dtype=torch.uint8, device=device)
    dist.all_gather_into_tensor(out, t, group=group)
    rows = out.cpu().view(world, IDENTITY_BYTES)
    return [json.loads(bytes(r.tolist()).rstrip(b"\0").decode()) for r in rows]
