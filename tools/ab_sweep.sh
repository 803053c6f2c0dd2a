#!/bin/bash
# Layout throughput A/B of alternative libp1hip.so builds (tools/sweep.py on
# a few message lengths per build).  usage: TAG=x SWEEP_LENGTHS=45,53 bash tools/ab_sweep.sh lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd); OUT=$ROOT/gpurun_out; TAG=${TAG:-abs}; mkdir -p "$OUT"
export SWEEP_LENGTHS=${SWEEP_LENGTHS:-8,45,53,54,63,100,109,120}
for lib in "$@"; do
  n=$(basename "$lib" .so)
  echo "== $n ($(date +%T))"
  P1HIP_LIB="$ROOT/$lib" timeout -k 10 300 python "$ROOT/tools/sweep.py" > "$OUT/${TAG}_$n.jsonl" 2> "$OUT/${TAG}_$n.err" || { echo "stopping: $n"; exit 1; }
done
echo "== done"
