"""ctypes binding of libp1hip.so (declarations: include/p1hip.h).

Fails loudly: a missing library, a missing symbol or a non-zero return code
raises P1HipError.  Nothing here computes a hash on the CPU.

A process that also uses torch on the GPU must import torch BEFORE the
library is loaded: the torch wheel ships its own HIP runtime, and
libp1hip.so has to bind to that copy; the other order leaves two HIP
runtimes in the process and the second to initialise sees no device.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

U64 = ctypes.c_uint64


class P1HipError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__(f"p1hip rc={rc}: {msg}")
        self.rc = rc


class Stats(ctypes.Structure):
    _fields_ = [
        ("scans", U64),
        ("fast_launches", U64),
        ("fast_nonces", U64),
        ("fast_alg_ops", U64),
        ("generic_launches", U64),
        ("generic_nonces", U64),
        ("scan_wall_ms", ctypes.c_double),
        ("scan_launches", U64),
        ("scan_nonces", U64),
        ("scan_alg_ops", U64),
        ("scan_kernel_ms", ctypes.c_double),
        ("small_scans", U64),
        ("table_replans", U64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class DeviceStats(ctypes.Structure):
    _fields_ = [
        ("ordinal", ctypes.c_int32),
        ("active", ctypes.c_int32),
        ("shard_first", U64),
        ("shard_last", U64),
        ("scans", U64),
        ("scan_launches", U64),
        ("scan_nonces", U64),
        ("scan_alg_ops", U64),
        ("scan_kernel_ms", ctypes.c_double),
        ("phase1_ms", ctypes.c_double),
        ("gather_ms", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class DeviceInfo(ctypes.Structure):
    _fields_ = [
        ("ordinal", ctypes.c_int32),
        ("cu_count", ctypes.c_int32),
        ("clock_khz", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("hbm_bytes", U64),
        ("pci_bus_id", ctypes.c_char * 32),
        ("arch", ctypes.c_char * 32),
        ("uuid", ctypes.c_ubyte * 16),
    ]

    def as_dict(self):
        return {"ordinal": self.ordinal, "cu_count": self.cu_count, "clock_khz": self.clock_khz,
                "hbm_bytes": self.hbm_bytes, "pci_bus_id": self.pci_bus_id.decode(errors="replace"),
                "arch": self.arch.decode(errors="replace"), "uuid": bytes(self.uuid).hex()}


def lib_path():
    # P1HIP_LIB selects an alternative build of the same library (A/B tuning
    # builds under p1_amd/variants/); default is the in-tree libp1hip.so.
    return os.environ.get("P1HIP_LIB") or os.path.join(_HERE, "libp1hip.so")


# (name, restype, argtypes) for every entry point of include/p1hip.h
SIGNATURES = [
    ("p1hip_init", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    ("p1hip_init_devices", ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    ("p1hip_scan", ctypes.c_int,
     [ctypes.c_char_p, ctypes.c_size_t, U64, U64, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
    ("p1hip_hash", ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, U64, ctypes.POINTER(U64)]),
    ("p1hip_plan_shards", ctypes.c_int,
     [ctypes.c_char_p, ctypes.c_size_t, U64, U64, ctypes.c_int, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
    ("p1hip_reduce_pairs", ctypes.c_int,
     [ctypes.POINTER(U64), ctypes.POINTER(U64), ctypes.c_size_t, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
    ("p1hip_set_profiling", ctypes.c_int, [ctypes.c_int]),
    ("p1hip_get_stats", ctypes.c_int, [ctypes.POINTER(Stats)]),
    ("p1hip_reset_stats", None, []),
    ("p1hip_get_device_stats", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(DeviceStats)]),
    ("p1hip_device_count", ctypes.c_int, []),
    ("p1hip_device_info", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(DeviceInfo)]),
    ("p1hip_comm_info", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("p1hip_abi_version", ctypes.c_int, []),
    ("p1hip_test_knobs", ctypes.c_char_p, []),
    ("p1hip_last_error", ctypes.c_char_p, []),
    ("p1hip_version", ctypes.c_char_p, []),
    ("p1hip_shutdown", None, []),
]


def load(path=None):
    """Load libp1hip.so (once).  Raises if it is missing or incomplete."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or lib_path()
    if not os.path.exists(p):
        raise P1HipError(-100, f"{p} not built (run `make` or __graft_entry__.build())")
    lib = ctypes.CDLL(p)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)  # AttributeError if the export is missing
        fn.restype = res
        fn.argtypes = args
    if lib.p1hip_abi_version() != ABI_VERSION:
        raise P1HipError(-100, f"{p}: ABI version {lib.p1hip_abi_version()}, this binding reads version "
                               f"{ABI_VERSION} structs (rebuild the library)")
    if path is None:
        _LIB = lib
    return lib


def _check(rc):
    if rc != 0:
        raise P1HipError(rc, load().p1hip_last_error().decode(errors="replace"))


def _bytes(msg):
    if isinstance(msg, str):
        return msg.encode("utf-8")  # Go strings are UTF-8 bytes after the JSON round trip
    return bytes(msg)


def init(want_devices=0):
    got = ctypes.c_int(0)
    _check(load().p1hip_init(int(want_devices), ctypes.byref(got)))
    return got.value


def init_devices(ordinals):
    arr = (ctypes.c_int * len(ordinals))(*ordinals)
    _check(load().p1hip_init_devices(arr, len(ordinals)))


def scan(msg, lower, upper):
    """miner.go:56-63 on the GPU: (min hash, its nonce) over [lower, upper]."""
    m = _bytes(msg)
    h, n = U64(), U64()
    _check(load().p1hip_scan(m, len(m), int(lower), int(upper), ctypes.byref(h), ctypes.byref(n)))
    return h.value, n.value


def hash(msg, nonce):  # noqa: A001 - mirrors bitcoin.Hash
    m = _bytes(msg)
    h = U64()
    _check(load().p1hip_hash(m, len(m), int(nonce), ctypes.byref(h)))
    return h.value


def plan_shards(msg, lower, upper, n):
    """p1hip_plan_shards: [lower, upper] cut into n contiguous shards of
    near-equal predicted GPU time; a list of inclusive (lo, hi) or None for
    an empty shard.  Host-only: needs the library, not a device."""
    m = _bytes(msg)
    first, last = (U64 * n)(), (U64 * n)()
    _check(load().p1hip_plan_shards(m, len(m), int(lower), int(upper), int(n), first, last))
    return [(a, b) if a <= b else None for a, b in zip(first, last)]


def reduce_pairs(hashes, nonces):
    n = len(hashes)
    assert n == len(nonces)
    ha = (U64 * max(n, 1))(*hashes)
    na = (U64 * max(n, 1))(*nonces)
    h, o = U64(), U64()
    _check(load().p1hip_reduce_pairs(ha, na, n, ctypes.byref(h), ctypes.byref(o)))
    return h.value, o.value


def set_profiling(on):
    _check(load().p1hip_set_profiling(1 if on else 0))


def get_stats():
    s = Stats()
    _check(load().p1hip_get_stats(ctypes.byref(s)))
    return s.as_dict()


def get_device_stats(index):
    """Per-device accounting since reset_stats (p1hip_get_device_stats)."""
    s = DeviceStats()
    _check(load().p1hip_get_device_stats(int(index), ctypes.byref(s)))
    return s.as_dict()


def device_info(index):
    """Identity of device `index` (p1hip_device_info): ordinal, PCI bus id,
    arch, CU count, clock, HBM bytes, UUID."""
    s = DeviceInfo()
    _check(load().p1hip_device_info(int(index), ctypes.byref(s)))
    return s.as_dict()


def comm_info(index):
    """(nranks, rank) of device `index`'s RCCL communicator as RCCL reports
    it (p1hip_comm_info: ncclCommCount / ncclCommUserRank); (0, -1) for a
    device without one."""
    n, r = ctypes.c_int(0), ctypes.c_int(-1)
    _check(load().p1hip_comm_info(int(index), ctypes.byref(n), ctypes.byref(r)))
    return n.value, r.value


# include/p1hip.h P1HIP_ABI_VERSION: the struct layouts this module declares
ABI_VERSION = 5


def abi_version():
    return load().p1hip_abi_version()


def test_knobs():
    """The library's test knobs in force for this process, as a dict ({} in
    production: the knobs are honoured only under P1HIP_TEST_KNOBS=1)."""
    raw = load().p1hip_test_knobs().decode()
    return dict(kv.split("=", 1) if "=" in kv else (kv, "?") for kv in raw.split(";") if kv)


def reset_stats():
    load().p1hip_reset_stats()


def device_count():
    return load().p1hip_device_count()


def shutdown():
    load().p1hip_shutdown()


def version():
    return load().p1hip_version().decode()


def codeobj_bytes(lib=None):
    """The gfx950 code object embedded in the library (the bytes between the
    p1hip_kernels_co / p1hip_kernels_co_end symbols of
    csrc/p1hip_kernels_blob.S, i.e. build/p1hip_kernels.hsaco as linked):
    the exact kernels every scan through this library runs."""
    lib = lib or load()
    start = ctypes.addressof(ctypes.c_char.in_dll(lib, "p1hip_kernels_co"))
    end = ctypes.addressof(ctypes.c_char.in_dll(lib, "p1hip_kernels_co_end"))
    if end <= start:
        raise P1HipError(-100, "embedded code object is empty")
    return ctypes.string_at(start, end - start)


def codeobj_sha256(lib=None):
    """sha256 (hex) of the embedded code object: the key that ties a rocprof
    or PMC summary under profiles/ to the kernels it measured."""
    import hashlib

    return hashlib.sha256(codeobj_bytes(lib)).hexdigest()
