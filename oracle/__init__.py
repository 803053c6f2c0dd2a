"""ORACLE -- test infrastructure only.

ctypes wrapper of oracle/libp1oracle.so, the CPU restatement of the
reference's hot path (hash.go:13-17, miner.go:56-63; see p1_oracle.c).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the reported CPU baseline.
The product (p1_amd, libp1hip.so) never imports it.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
U64 = ctypes.c_uint64


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _LIB
    if _LIB is None:
        p = os.path.join(_HERE, "libp1oracle.so")
        if not os.path.exists(p):
            build()
        lib = ctypes.CDLL(p)
        lib.p1o_hash.restype = U64
        lib.p1o_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64]
        lib.p1o_scan.restype = ctypes.c_int
        lib.p1o_scan.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64, U64,
                                 ctypes.POINTER(U64), ctypes.POINTER(U64)]
        lib.p1o_scan_mt.restype = ctypes.c_int
        lib.p1o_scan_mt.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64, U64, ctypes.c_int,
                                    ctypes.POINTER(U64), ctypes.POINTER(U64)]
        lib.p1o_sha256.restype = None
        lib.p1o_sha256.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        _LIB = lib
    return _LIB


def _b(msg):
    return msg.encode("utf-8") if isinstance(msg, str) else bytes(msg)


def sha256(data):
    out = ctypes.create_string_buffer(32)
    d = _b(data)
    load().p1o_sha256(d, len(d), out)
    return out.raw


def hash(msg, nonce):  # noqa: A001 - mirrors bitcoin.Hash
    m = _b(msg)
    return load().p1o_hash(m, len(m), int(nonce))


def scan(msg, lower, upper, threads=1):
    m = _b(msg)
    h, n = U64(), U64()
    if threads > 1:
        rc = load().p1o_scan_mt(m, len(m), int(lower), int(upper), int(threads), ctypes.byref(h), ctypes.byref(n))
    else:
        rc = load().p1o_scan(m, len(m), int(lower), int(upper), ctypes.byref(h), ctypes.byref(n))
    if rc != 0:
        raise RuntimeError("oracle scan failed")
    return h.value, n.value
