"""configs[4]-style end-to-end run without the LSP transport: p1server splits
one [0, 2^36) job for 'bradfitz' into chunks and deals them to N GPU-backed
miner processes (`p1miner serve --device i`), then prints one JSON line with
the wall-clock throughput and the result.  On a 1-GPU box all miners share
device 0."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    miners = int(os.environ.get("MINERS", "1"))
    ngpu = int(os.environ.get("NGPU", "1"))
    hi = int(os.environ.get("UPPER", str((1 << 36) - 1)))
    chunk = int(os.environ.get("CHUNK", str(1 << 32)))
    devs = ",".join(str(i % ngpu) for i in range(miners))
    cmd = [os.path.join(ROOT, "p1_amd", "p1server"), "--miners", str(miners), "--devices", devs,
           "--chunk", str(chunk), "scan", "bradfitz", "0", str(hi)]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=1200)
    dt = time.perf_counter() - t0
    out = {"workload": f"p1server: 'bradfitz' [0, {hi}] in chunks of {chunk} over {miners} miner processes "
                       f"on {ngpu} GPU(s), stdio transport (LSP out of scope)",
           "rc": r.returncode, "stdout": r.stdout.strip(), "wall_s": dt,
           "GH_s_incl_startup": (hi + 1) / dt / 1e9}
    print(json.dumps(out))
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
