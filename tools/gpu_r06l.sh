#!/bin/bash
# r06l: the shipped work-queue build against the same source compiled with
# MachineLICM off (nolicm: no round constants hoisted out of the tile loop,
# 19 instead of 226 SGPR spills, but the K materialisation stays in the
# per-nonce loops) and the static grid: c2/c3/c4 through tools/gpu_ab.sh,
# then the MODE 5/7 layouts through tools/sweep.py (results re-hashed).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
TAG=r06l LIBS="p1_amd/variants/libp1hip_nolicm.so p1_amd/variants/libp1hip_static.so" C4STEPS=2 C3STEPS=3 \
  timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r06l_ab.log 2>&1 || exit $?
export SWEEP_LENGTHS=54,112,124,113,8,120
for run in base nolicm static base2; do
  case $run in base*) lib=p1_amd/libp1hip.so ;; *) lib=p1_amd/variants/libp1hip_$run.so ;; esac
  P1HIP_LIB="$PWD/$lib" timeout -k 10 300 python tools/sweep.py > gpurun_out/r06l_sweep_$run.jsonl 2> gpurun_out/r06l_sweep_$run.err || exit $?
done
