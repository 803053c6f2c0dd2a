#!/bin/bash
# A/B throughput of alternative builds of libp1hip.so on one GPU box.
# usage: TAG=r01k bash tools/ab_variants.sh p1_amd/variants/libp1hip_X.so ...
# Runs the default build first and last (drift check), each variant in
# between; every run is bench.py --steps 5 --warmup 1 --no-cpu under its own
# time limit.  Stops at the first run that does not exit 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-ab}
ARGS=${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu}
mkdir -p "$OUT"
run() {  # run <name> <lib or empty>
  echo "== $1 ($(date +%T))"
  P1HIP_LIB=$2 timeout -k 10 300 python "$ROOT/bench.py" $ARGS > "$OUT/${TAG}_$1.json" 2> "$OUT/${TAG}_$1.err"
  local rc=$?
  python3 -c "import json,sys
for l in open('$OUT/${TAG}_$1.json'):
    if l.startswith('{'):
        d=json.loads(l); print(json.dumps({'name':'$1','value':d['value'],'kernel_GH_s':d['roofline']['kernel_hashes_per_s_G'],'ok':d['result']['matches_known']}))" | tee -a "$OUT/${TAG}_summary.jsonl"
  [ $rc -eq 0 ] || { echo "stopping: $1 rc=$rc"; exit $rc; }
}
run base ""
for lib in "$@"; do run "$(basename "$lib" .so)" "$ROOT/$lib"; done
run base_end ""
echo "== done"
