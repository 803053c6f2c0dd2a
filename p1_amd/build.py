"""Build-if-missing for fresh checkouts (the GPU box has hipcc too).

Everything is normally prebuilt by `make` / __graft_entry__.build(); this
only runs make when an artefact is absent, under a file lock so that
several torchrun ranks starting together build once."""
import fcntl
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARTEFACTS = ["p1_amd/libp1hip.so", "oracle/libp1oracle.so", "p1_amd/p1miner", "p1_amd/p1server", "p1_amd/p1client",
             "tools/p1emu", "tools/lsp_scenarios", "tools/lsp_fake_miner", "tools/libp1clock.so"]


def missing():
    return [a for a in ARTEFACTS if not os.path.exists(os.path.join(ROOT, a))]


def ensure_built():
    if not missing():
        return
    lock = os.path.join(ROOT, ".build.lock")
    with open(lock, "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        try:
            if missing():
                jobs = str(min(16, os.cpu_count() or 1))
                subprocess.run(["make", "-C", ROOT, "-j", jobs, "all"], check=True)
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)
