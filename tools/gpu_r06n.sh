#!/bin/bash
# r06n: the shipped build against the same source compiled without
# MachineLICM and passed through isa_post --hoist-consts (nolicmh: the
# round constants hoisted by the post-pass out of the per-nonce loops only)
# and the static grid: a 60 s randomized parity stress of nolicmh first,
# then c2/c3/c4 through tools/gpu_ab.sh and layouts through tools/sweep.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
P1HIP_LIB="$PWD/p1_amd/variants/libp1hip_nolicmh.so" timeout -k 10 200 python tools/stress.py 60 > gpurun_out/r06n_stress_nolicmh.json 2> gpurun_out/r06n_stress_nolicmh.err || exit $?
TAG=r06n LIBS="p1_amd/variants/libp1hip_nolicmh.so p1_amd/variants/libp1hip_static.so" C4STEPS=2 C3STEPS=3 \
  timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r06n_ab.log 2>&1 || exit $?
export SWEEP_LENGTHS=54,112,124,113,8,120,43
for run in base nolicmh static base2; do
  case $run in base*) lib=p1_amd/libp1hip.so ;; *) lib=p1_amd/variants/libp1hip_$run.so ;; esac
  P1HIP_LIB="$PWD/$lib" timeout -k 10 300 python tools/sweep.py > gpurun_out/r06n_sweep_$run.jsonl 2> gpurun_out/r06n_sweep_$run.err || exit $?
done
