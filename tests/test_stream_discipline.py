"""Every device operation of libp1hip.so goes to the library's own stream.

Why (DESIGN.md "Small scans"): a null-stream call such
as a synchronous hipMemset gives the process a second hardware queue.  With 8
`p1miner` processes on one GPU plus a parent holding RCCL queues, the
miners' kernels were never scheduled (configs[4] test hung until the ticket
reset moved to hipMemsetAsync on d.stream).  This CPU test reads
p1_amd/csrc/p1hip.hip and fails on any HIP call outside an allow-list of
stream-free management calls, and on any stream-taking call whose stream is
not the device's own `d.stream` -- so a later null-stream call cannot bring
the hang back unnoticed.  The queue count itself is observed on the GPU in
tests/test_lsp_bitcoin.py (configs[4] over LSP)."""
import os
import re

from conftest import ROOT

SRC = os.path.join(ROOT, "p1_amd", "csrc", "p1hip.hip")

# host-side management calls that enqueue nothing on any stream
STREAM_FREE = {
    "hipDeviceGetPCIBusId", "hipEventCreate", "hipEventDestroy", "hipEventElapsedTime", "hipEventSynchronize", "hipFree",
    "hipGetDeviceCount", "hipGetDeviceProperties", "hipGetErrorString", "hipGetLastError", "hipHostFree",
    "hipHostMalloc", "hipMalloc", "hipModuleGetFunction", "hipModuleLoadData", "hipModuleUnload",
    "hipModuleOccupancyMaxActiveBlocksPerMultiprocessor",  # k_scan's grid (a query of the function's resources)
    "hipSetDevice", "hipStreamCreateWithFlags", "hipStreamDestroy", "hipStreamSynchronize",
}
# calls that enqueue work: their stream argument (last) must be the device's
STREAM_ARG = {"hipMemcpyAsync", "hipMemsetAsync", "hipEventRecord", "ncclAllGather", "launch",
              "hipModuleLaunchKernel"}


def _strip_comments(src):
    """Comments and string literals out (error messages name calls too)."""
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return re.sub(r'"(?:[^"\\\n]|\\.)*"', '""', src)


def _calls(src, name):
    """(line, [args]) of every call `name(...)`, arguments split at top level."""
    out = []
    for m in re.finditer(r"\b" + re.escape(name) + r"\s*\(", src):
        i, depth, cur, args = m.end(), 1, "", []
        while depth:
            c = src[i]
            if c in "([{":
                depth += 1
            elif c in ")]}":
                depth -= 1
            if depth == 1 and c == ",":
                args.append(cur.strip())
                cur = ""
            elif depth:
                cur += c
            i += 1
        args.append(cur.strip())
        out.append((src.count("\n", 0, m.start()) + 1, args))
    return out


def test_only_allowed_hip_calls():
    src = _strip_comments(open(SRC).read())
    used = set(re.findall(r"\b(hip[A-Z]\w*)\s*\(", src))
    unknown = used - STREAM_FREE - STREAM_ARG
    assert not unknown, f"HIP calls outside the allow-list (null stream / synchronous?): {sorted(unknown)}"
    assert "<<<" not in src and "hipLaunchKernelGGL" not in src


def test_every_enqueue_names_the_device_stream():
    src = _strip_comments(open(SRC).read())
    seen = 0
    for name in sorted(STREAM_ARG):
        for line, args in _calls(src, name):
            if name == "launch" and args[0].startswith("hipFunction_t"):
                continue  # the template's own definition
            if name == "hipModuleLaunchKernel":
                # only inside the launch() template, which forwards its `st`
                assert args[8] == "st", (line, args)
                continue
            stream = args[3] if name == "launch" else args[-1]
            assert stream == "d.stream", f"p1hip.hip:{line}: {name} on stream '{stream}'"
            seen += 1
    assert seen >= 20  # the checker really parsed the calls


def test_host_programs_make_no_hip_calls():
    # the miner/server/client reach the GPU only through the C ABI
    for fn in os.listdir(os.path.join(ROOT, "p1_amd", "host")):
        if fn.endswith((".cpp", ".hpp")):
            src = _strip_comments(open(os.path.join(ROOT, "p1_amd", "host", fn)).read())
            assert not re.search(r"\bhip[A-Z]\w*\s*\(", src), fn
