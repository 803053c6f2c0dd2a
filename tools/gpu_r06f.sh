#!/bin/bash
# r06f: the MODE 5 / MODE 7 layouts whose sweep rate moved between r05af and
# r06e, on the work-queue build and the static-grid variant, same box,
# alternating (tools/sweep.py, every result re-hashed on the oracle).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export SWEEP_LENGTHS=54,112,48,118,124,113,119,49,8,43
for run in wq static wq2 static2; do
  case $run in wq*) lib=p1_amd/libp1hip.so ;; *) lib=p1_amd/variants/libp1hip_static.so ;; esac
  P1HIP_LIB="$PWD/$lib" timeout -k 10 300 python tools/sweep.py > gpurun_out/r06f_sweep_$run.jsonl 2> gpurun_out/r06f_sweep_$run.err || exit $?
done
