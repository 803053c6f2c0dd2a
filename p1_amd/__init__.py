"""p1_amd -- MI355X (gfx950) drop-in for the bitcoin miner's nonce scan.

The product is the C-ABI library ``p1_amd/libp1hip.so`` (include/p1hip.h).
This package is thin Python plumbing over it (ctypes), used by bench.py and
the tests.  There is no CPU fallback: every call goes to the HIP kernels and
raises if the library or a gfx950 device is missing.

Reference seam: /root/reference/src/github.com/cmu440/bitcoin/miner/miner.go:56-63.
"""
from ._lib import (  # noqa: F401
    P1HipError,
    lib_path,
    load,
    init,
    init_devices,
    scan,
    hash,
    reduce_pairs,
    plan_shards,
    set_profiling,
    get_stats,
    get_device_stats,
    reset_stats,
    device_count,
    device_info,
    comm_info,
    abi_version,
    ABI_VERSION,
    test_knobs,
    shutdown,
    version,
    codeobj_bytes,
    codeobj_sha256,
)
from .sharding import shard_range, combine_keys  # noqa: F401
