set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06c_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_gpu_small.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06c_pytest_gpu.log 2>&1 || exit $?
TAG=r06c LIBS="p1_amd/variants/libp1hip_static.so" C4STEPS=3 C3STEPS=3 timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/r06c_ab.log 2>&1
