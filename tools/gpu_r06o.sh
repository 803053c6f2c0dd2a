#!/bin/bash
# r06o: longer randomized parity stress on the shipped code object:
# production settings 300 s, the fast variants forced onto small ranges
# 300 s, and messages of 0..2000 bytes (up to 31 midstate blocks) 150 s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 400 python tools/stress.py 300 640 > gpurun_out/r06o_stress.json 2> gpurun_out/r06o_stress.err || exit $?
P1HIP_TEST_KNOBS=1 P1HIP_MIN_FAST_THREADS=1 P1HIP_SMALL_MAX_NONCES=0 timeout -k 10 400 python tools/stress.py 300 641 > gpurun_out/r06o_stress_k3.json 2> gpurun_out/r06o_stress_k3.err || exit $?
STRESS_MAXLEN=2000 timeout -k 10 250 python tools/stress.py 150 642 > gpurun_out/r06o_stress_long.json 2> gpurun_out/r06o_stress_long.err || exit $?
