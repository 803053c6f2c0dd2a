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


def _stats_worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    import oracle
    from p1_amd.dist import distributed_scan, gather_rank_identity, gather_rank_stats

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    timing = {}
    for _ in range(3):
        distributed_scan(b"bradfitz", 0, 9999, oracle.scan, timing=timing)
    mine = {"shard_lo": timing["shard"][0], "shard_hi": (1 << 64) - 1 - rank, "nonces": rank + 1,
            "launches": 2 * rank, "alg_ops": (1 << 63) + rank, "kernel_ms": 1.5 * rank,
            "scan_ms": timing["scan_s"] * 1e3, "gather_ms": timing["gather_s"] * 1e3, "elapsed_ms": 10.0 + rank,
            "step_ms_median": 3.25}
    got = gather_rank_stats(mine)
    ident = gather_rank_identity({"hostname": "host-" + "é" * rank, "ordinal": rank, "pci_bus_id": f"0000:{rank:02x}:00.0",
                                  "uuid": f"{rank:032x}", "rank": rank})
    dist.destroy_process_group()
    q.put((rank, timing["steps"], timing["shard"], got, ident))


@pytest.mark.parametrize("world", [2, 3])
def test_gather_rank_stats_gloo(world):
    """bench.py's N>1 diagnostics: every rank's shard, kernel and collective
    time reach rank 0 intact (u64 values above 2^63 included)."""
    from p1_amd import shard_range

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, steps, shard, got, ident in res:
        # bench.py's per-rank device identity: one record per rank, in rank order
        assert [i["rank"] for i in ident] == list(range(world))
        assert [i["pci_bus_id"] for i in ident] == [f"0000:{r:02x}:00.0" for r in range(world)]
        assert ident[world - 1]["hostname"] == "host-" + "é" * (world - 1)
        assert steps == 3 and tuple(shard) == shard_range(0, 9999, rank, world)
        assert len(got) == world
        for r, g in enumerate(got):
            assert g["rank"] == r
            assert g["shard_lo"] == shard_range(0, 9999, r, world)[0]
            assert g["shard_hi"] == (1 << 64) - 1 - r and g["alg_ops"] == (1 << 63) + r
            assert g["nonces"] == r + 1 and g["launches"] == 2 * r
            assert g["kernel_ms"] == 1.5 * r and g["elapsed_ms"] == 10.0 + r and g["step_ms_median"] == 3.25
            assert g["gather_ms"] >= 0.0 and g["scan_ms"] > 0.0
