#!/bin/bash
# One GPU-box session: VALU micro-benchmark, GPU parity tests, bench, rocprof.
# Each GPU step has its own time limit.  A test FAILURE (exit 1) does not stop
# the session; any fault/abort/timeout (other non-zero codes) ends it at once.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-r01}
mkdir -p "$OUT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_PEAK:-0}" = 1 ] || step valu_peak 120 "$ROOT/tools/valu_peak" > "$OUT/${TAG}_valu_peak.jsonl"
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -m pytest "$ROOT/tests" -m gpu -x -q -p no:cacheprovider > "$OUT/${TAG}_pytest_gpu.log" 2>&1
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import sys; sys.path.insert(0, '$ROOT'); import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1
step bench 600 python "$ROOT/bench.py" ${BENCH_ARGS:-} > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu
fi
echo "== done"
