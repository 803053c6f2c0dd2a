#!/bin/bash
# The host programs under sanitizers (CPU only; no GPU code is built or run).
#
#   tools/sanitize.sh [out.json]
#
# Builds `make sanitize` (ASan+UBSan and TSan builds of the LSP stack, the
# server, the client, the CPU test-double miner and the scheduler unit test)
# and, when present, build/san/asan/p1emu (`make sanitize-emu`, ~6 min: the
# planner + every kernel variant replayed on the host).  Then re-runs the
# CPU tests that drive those programs with P1_SAN_DIR pointing at each build
# (tests/conftest.py host_bin) and every sanitizer writing its reports to
# files: a run passes only if pytest passes AND no report file appears (a
# miner or server launched in the background has no exit code to check).
set -u
cd "$(dirname "$0")/.."
OUT=${1:-}
make -s sanitize >/dev/null || { echo "sanitize: build failed"; exit 2; }
RES=()
status=0
for san in asan tsan; do
  logs=$(mktemp -d /tmp/p1san_${san}_XXXX)
  export P1_SAN_DIR=$PWD/build/san/$san
  export ASAN_OPTIONS="detect_leaks=1:log_path=$logs/asan"
  export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:log_path=$logs/ubsan"
  export TSAN_OPTIONS="halt_on_error=0:log_path=$logs/tsan"
  tests="tests/test_lsp.py tests/test_lsp_bitcoin.py tests/test_server.py"
  if [ "$san" = asan ] && [ -x build/san/asan/p1emu ]; then
    tests="$tests tests/test_host_logic.py"
  fi
  t0=$(date +%s)
  python3 -m pytest $tests -q -m "not gpu" -n 4 -p no:cacheprovider > "$logs/pytest.txt" 2>&1
  rc=$?
  # the scheduler unit test on its own (single-threaded: ASan/UBSan is what it needs)
  if [ "$san" = asan ]; then
    "$P1_SAN_DIR/sched_test" > "$logs/sched.txt" 2>&1 || rc=1
  fi
  reports=$(ls "$logs" | grep -E '^(asan|ubsan|tsan)\.' | wc -l)
  summary=$(tail -1 "$logs/pytest.txt")
  echo "$san: pytest rc=$rc ($summary), sanitizer report files: $reports, logs in $logs"
  [ "$rc" -eq 0 ] && [ "$reports" -eq 0 ] || status=1
  RES+=("{\"sanitizer\": \"$san\", \"tests\": \"$tests\", \"pytest_rc\": $rc, \"pytest\": \"$summary\", \"report_files\": $reports, \"seconds\": $(( $(date +%s) - t0 )), \"p1emu\": $([ "$san" = asan ] && [ -x build/san/asan/p1emu ] && echo true || echo false)}")
done
if [ -n "$OUT" ]; then
  printf '%s\n' "${RES[@]}" > "$OUT"
fi
exit $status
