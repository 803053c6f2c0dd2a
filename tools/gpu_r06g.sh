#!/bin/bash
# r06g: the same work-queue code object with the queue (default grid) and
# without it (P1HIP_SCAN_GRID at 2^22: one tile per workgroup, the round-5
# dispatch), alternating on one box, on the layouts whose rate moved in r06f
# (tools/sweep.py, every result re-hashed on the oracle).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export SWEEP_LENGTHS=${SWEEP_LENGTHS:-54,112,48,118,124,113,119,49,8,120}
for run in q grid q2 grid2; do
  case $run in q*) g=0 ;; *) g=4194304 ;; esac
  P1HIP_TEST_KNOBS=1 P1HIP_SCAN_GRID=$g timeout -k 10 300 python tools/sweep.py > gpurun_out/r06g_sweep_$run.jsonl 2> gpurun_out/r06g_sweep_$run.err || exit $?
done
