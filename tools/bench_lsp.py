"""configs[4] end to end over LSP/UDP: `p1server lsp` splits one 'bradfitz'
[0, 2^36) request into chunks and deals them to N GPU-backed miner processes
(`p1miner lsp --device i`), all with the LSP window and write-drop knobs of
configs[4] (window 8, 5% of every write dropped in every process).  A first
request warms every miner (device init, code object, first launch); then
REPS requests are timed from the client's start to its Result line.  Prints
one JSON line.  On a 1-GPU box all miners share device 0, so the number is
the system's overhead on top of one GPU, not an 8-GPU rate.

env: MINERS (8), NGPU (1), UPPER (2^36 - 1), CHUNK (2^32), WINDOW (8),
     DROP (5), REPS (3), EPOCH_MS (unset: the reference's 2000 ms epochs;
     a lost datagram is resent one epoch later, so at 5% drop the wall time
     holds whole epochs), COPIES (unset: the programs' default,
     lsp::DefaultAppCopies = 3; 1 = the reference protocol: datagrams per
     first transmission), CONNECT_COPIES (unset: the programs' default
     1, the reference's single Connect per attempt; lsp::Params::
     ConnectCopies); FAKE=1 runs the CPU oracle-backed miner double
     (tools/lsp_fake_miner, test plumbing only) instead of p1miner
Reference: server.go:45-170 (dispatch), miner.go:13-73, client.go:21."""
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERVER = os.path.join(ROOT, "p1_amd", "p1server")
MINER = os.path.join(ROOT, "p1_amd", "p1miner")
CLIENT = os.path.join(ROOT, "p1_amd", "p1client")
FAKE = os.path.join(ROOT, "tools", "lsp_fake_miner")


def known(upper):
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        for v in json.load(f)["scan"]:
            if v.get("large") and v["msg_hex"] == b"bradfitz".hex() and v["lower"] == 0 and v["upper"] == upper:
                return [v["hash"], v["nonce"]]
    return None


def main():
    miners = int(os.environ.get("MINERS", "8"))
    ngpu = int(os.environ.get("NGPU", "1"))
    upper = int(os.environ.get("UPPER", str((1 << 36) - 1)))
    chunk = int(os.environ.get("CHUNK", str(1 << 32)))
    window = os.environ.get("WINDOW", "8")
    drop = os.environ.get("DROP", "5")
    reps = int(os.environ.get("REPS", "3"))
    env = dict(os.environ, P1LSP_WRITE_DROP=drop)
    lsp = ["--window", window]
    epoch = os.environ.get("EPOCH_MS")
    if epoch:
        lsp += ["--epoch-millis", epoch]
    copies = os.environ.get("COPIES")
    if copies:
        lsp += ["--copies", copies]
    cc = os.environ.get("CONNECT_COPIES")
    # the server never sends a Connect: only miners and the client take it
    peer = ["--connect-copies", cc] if cc else []
    procs = []
    try:
        srv = subprocess.Popen([SERVER, "--chunk", str(chunk)] + lsp + ["lsp", "0"],
                               stdout=subprocess.PIPE, text=True, env=env)
        procs.append(srv)
        line = srv.stdout.readline()
        if not line.startswith("Server listening on port"):
            raise SystemExit(f"bench_lsp: server said {line!r}")
        hp = f"127.0.0.1:{int(line.split()[-1])}"
        fake = os.environ.get("FAKE") == "1"
        for i in range(miners):
            argv = [FAKE, hp] + lsp + peer if fake else [MINER, "lsp", hp, "--device", str(i % ngpu)] + lsp + peer
            procs.append(subprocess.Popen(argv, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env))

        time.sleep(0.5)
        dead = [p.args for p in procs[1:] if p.poll() is not None]
        if dead:
            raise SystemExit(f"bench_lsp: miner exited at start: {dead[0]}")

        def request():
            t0 = time.perf_counter()
            r = subprocess.run([CLIENT, hp, "bradfitz", str(upper)] + lsp + peer, capture_output=True, text=True,
                               timeout=600, env=env)
            dt = time.perf_counter() - t0
            if r.returncode != 0 or not r.stdout.startswith("Result"):
                raise SystemExit(f"bench_lsp: client rc={r.returncode} out={r.stdout!r} err={r.stderr[-500:]!r}")
            _, h, n = r.stdout.split()
            return dt, [int(h), int(n)]

        warm_s, _ = request()
        walls, results = [], []
        for _ in range(reps):
            dt, res = request()
            walls.append(dt)
            results.append(res)
        want = known(upper)
        med = statistics.median(walls)
        print(json.dumps({
            "workload": f"configs[4]: client 'bradfitz' maxNonce {upper} -> p1server lsp (chunks of {chunk}) -> "
                        f"{miners} {'CPU oracle miner doubles' if fake else f'p1miner lsp processes on {ngpu} GPU(s)'}"
                        f"; LSP window {window}, {drop}% write drop in every process, "
                        f"{epoch or 'default (2000)'} ms epochs, "
                        f"{copies or 'default (3)'} copies per first Data transmission, "
                        f"{cc or 'default (1)'} per Connect",
            "copies": int(copies) if copies else 3, "connect_copies": int(cc) if cc else 1, "epoch_ms": int(epoch) if epoch else 2000, "miners": miners,
            "reps": reps, "wall_s": walls, "wall_s_median": med, "wall_s_max": max(walls),
            "wall_s_p90": sorted(walls)[min(len(walls) - 1, int(0.9 * len(walls)))], "warmup_wall_s": warm_s,
            "GH_s": (upper + 1) / med / 1e9,
            "result": results[-1], "consistent": all(r == results[0] for r in results),
            "matches_known": (results[-1] == want) if want else None}), flush=True)
        if want and results[-1] != want:
            sys.exit(3)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()


if __name__ == "__main__":
    main()
