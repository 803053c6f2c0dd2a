"""One-process-per-GPU scan: contiguous shard per rank, 16-byte per-rank
results all-gathered over torch.distributed (backend "nccl" = RCCL over
xGMI on MI355X; "gloo" in the CPU tests), lexicographic (hash, nonce) min.

This is the only collective on the path: the reference has
no exchange step besides the final min of miner.go:56-63.
"""
import torch
import torch.distributed as dist

from .sharding import combine_keys, shard_range


def _to_i64(v):
    return v - (1 << 64) if v >= (1 << 63) else v


def _to_u64(v):
    return v + (1 << 64) if v < 0 else v


def distributed_scan(msg, lower, upper, scan_fn, device=None, group=None, shard_fn=None):
    """Scan [lower, upper] with every rank of `group` taking one contiguous
    shard through scan_fn(msg, lo, hi) -> (hash, nonce); returns the global
    result on every rank.

    shard_fn(msg, lower, upper, world) -> [(lo, hi) | None] * world picks the
    shards (default: equal nonce counts, sharding.shard_range); the GPU path
    passes p1_amd.plan_shards, the library's cost-balanced contiguous split.
    Every rank must use the same shard_fn."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if shard_fn is None:
        s = shard_range(lower, upper, rank, world)
    else:
        s = shard_fn(msg, lower, upper, world)[rank]
    key = scan_fn(msg, s[0], s[1]) if s is not None else (2**64 - 1, 0)
    t = torch.tensor([_to_i64(key[0]), _to_i64(key[1])], dtype=torch.int64, device=device)
    out = torch.empty(2 * world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out, t, group=group)
    v = [_to_u64(x) for x in out.tolist()]
    return combine_keys(list(zip(v[0::2], v[1::2])))
