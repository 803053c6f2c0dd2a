#!/bin/bash
# try to reproduce the r04p teardown abort -- the ASan
# stress driver for the r04p duration, through the NORMAL exit path
# (P1_SAN_NORMAL_EXIT=1), every ASan report symbolized into gpurun_out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=$PWD/gpurun_out
TAG=${TAG:-r05b}
S=${SAN_STRESS_S:-360}
mkdir -p "$OUT"
timeout -k 10 600 make -s -C "$PWD" -j16 sanitize-lib || exit $?
echo "== san_stress_normal_exit ${S}s ($(date +%T))"
P1_SAN_NORMAL_EXIT=1 ASAN_OPTIONS="detect_leaks=0:log_path=$OUT/${TAG}_asan_normal_exit" \
  ASAN_SYMBOLIZER_PATH=/opt/rocm/lib/llvm/bin/llvm-symbolizer \
  timeout -k 10 $((S + 240)) "$PWD/tools/san/capi_san_stress" "$S" > "$OUT/${TAG}_san_stress_normal_exit_${S}s.out" 2>&1
rc=$?
echo "== rc=$rc ($(date +%T))"
tail -3 "$OUT/${TAG}_san_stress_normal_exit_${S}s.out"
ls "$OUT" | grep "${TAG}_asan" || echo "no ASan report file"
exit 0
