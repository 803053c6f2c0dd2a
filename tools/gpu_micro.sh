#!/bin/bash
# Run an issue-rate microbenchmark (tools/dual, tools/loopbench: generated
# by tools/gen_dual.py, tools/gen_loopbench.py) and one PMC pass over it for
# the dual-issue count (SQ_ACTIVE_INST_VALU2) per kernel.
# usage: TAG=r05d tools/gpu_micro.sh BIN [BIN ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-r05}
mkdir -p "$OUT"
for b in "$@"; do
  echo "== $b ($(date +%T))"
  timeout -k 10 300 "$ROOT/tools/$b" > "$OUT/${TAG}_$b.jsonl" || exit $?
done
cd /tmp && export TMPDIR=/tmp
for b in "$@"; do
  echo "== $b pmc ($(date +%T))"
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVES GRBM_GUI_ACTIVE -d "$OUT/${TAG}_${b}pmc" -o pmc --output-format csv -- "$ROOT/tools/$b" > /dev/null || exit $?
done
echo "== micro done"
