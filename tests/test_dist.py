"""The N>1 path of bench.py on CPU: world_size-2 (and 3) gloo process
groups, contiguous shards, all-gather of the 16-byte results, lexicographic
min -- with the oracle standing in for the per-rank GPU scan."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cases, q, planned=False):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    import oracle
    from p1_amd.dist import distributed_scan

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def scan_fn(m, lo, hi):
        calls.append((lo, hi))
        return oracle.scan(m, lo, hi)

    shard_fn = None
    if planned:
        import p1_amd

        shard_fn = p1_amd.plan_shards  # host-only library call: no device needed
    out = [distributed_scan(m, lo, hi, scan_fn, shard_fn=shard_fn) for m, lo, hi in cases]
    dist.destroy_process_group()
    q.put((rank, out, calls))


@pytest.mark.parametrize("planned", [False, True], ids=["equal", "plan_shards"])
@pytest.mark.parametrize("world", [2, 3])
def test_distributed_scan_gloo(world, planned, oracle_mod):
    cases = [(b"bradfitz", 0, 9999), (b"msg", 0, 2), (b"x" * 70, 10**9 - 2000, 10**9 + 2000),
             (b"bradfitz", 5, 3), (b"msg", 0, 0)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q, planned)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [oracle_mod.scan(m, lo, hi) for m, lo, hi in cases]
    for rank, out, calls in res:
        assert out == want, rank
        # every rank scanned exactly its own contiguous shard
        from p1_amd import plan_shards, shard_range

        exp = [plan_shards(m, lo, hi, world)[rank] if planned else shard_range(lo, hi, rank, world)
               for m, lo, hi in cases]
        assert calls == [e for e in exp if e is not None]
