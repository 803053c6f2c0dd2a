#!/bin/bash
# Longer run of a fuzzer (CPU only): fuzz_codecs (tests/fuzz/fuzz_codecs.cpp,
# the wire codecs; default) or fuzz_planner (tests/fuzz/fuzz_planner.cpp).
#   tools/fuzz.sh [seconds] [jobs] [out.txt] [fuzz_codecs|fuzz_planner]
# Starts from tests/fuzz/seeds (codecs) or an empty corpus (planner) in a
# scratch directory; prints libFuzzer's final stats; exits non-zero on any
# crash, sanitizer report or property failure.
set -u
cd "$(dirname "$0")/.."
SECS=${1:-600}
JOBS=${2:-4}
OUT=${3:-/dev/stdout}
case "$OUT" in /*) ;; *) OUT="$PWD/$OUT" ;; esac
TARGET=${4:-fuzz_codecs}
make -s fuzz >/dev/null || exit 2
work=$(mktemp -d /tmp/p1fuzz_XXXX)
if [ "$TARGET" = fuzz_codecs ]; then cp -r tests/fuzz/seeds "$work/corpus"; else mkdir "$work/corpus"; fi
cd "$work"
rc=0
for j in $(seq 1 "$JOBS"); do
  "$OLDPWD/build/san/$TARGET" -max_total_time="$SECS" -print_final_stats=1 -max_len=4096 -seed=$((440 + j)) \
      corpus > "job$j.log" 2>&1 &
done
for j in $(seq 1 "$JOBS"); do wait -n || rc=1; done
{
  echo "$TARGET: $JOBS jobs x $SECS s, shared corpus (ASan + UBSan)"
  for j in $(seq 1 "$JOBS"); do
    echo "job $j: $(grep -E '^stat::number_of_executed_units' job$j.log | awk '{print $2}') runs," \
         "$(grep -E '^stat::new_units_added' job$j.log | awk '{print $2}') new units," \
         "peak rss $(grep -E '^stat::peak_rss_mb' job$j.log | awk '{print $2}') MB," \
         "crashes: $(ls crash-* leak-* timeout-* oom-* 2>/dev/null | wc -l)"
  done
  echo "corpus: $(ls corpus | wc -l) inputs; rc=$rc"
} > "$OUT"
[ "$rc" -eq 0 ] && ! ls crash-* leak-* timeout-* oom-* >/dev/null 2>&1
