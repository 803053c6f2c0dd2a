#!/bin/bash
# r06h: A/B of the work-queue build with the extended post-pass (default
# library), the same object through the round-6 first post-pass (wq1)
# library), and the round-5-shaped static grid:
# c2/c3/c4 through tools/gpu_ab.sh, then the MODE 5/7 and TRAIL layouts
# through tools/sweep.py per library (every result re-hashed).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
TAG=r06h LIBS="p1_amd/variants/libp1hip_wq1.so p1_amd/variants/libp1hip_static.so" C4STEPS=2 C3STEPS=3 \
  timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r06h_ab.log 2>&1 || exit $?
export SWEEP_LENGTHS=54,112,124,113,119,43,8,120
for run in base wq1 static base2; do
  case $run in base*) lib=p1_amd/libp1hip.so ;; *) lib=p1_amd/variants/libp1hip_$run.so ;; esac
  P1HIP_LIB="$PWD/$lib" timeout -k 10 300 python tools/sweep.py > gpurun_out/r06h_sweep_$run.jsonl 2> gpurun_out/r06h_sweep_$run.err || exit $?
done
