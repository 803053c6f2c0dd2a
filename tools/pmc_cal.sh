#!/bin/bash
# WRITE_SIZE / FETCH_SIZE calibration for k_scan's traffic (tools/wcal.hip)
# and repeat passes of the same counters on the bench's k_scan launch, one
# counter per rocprofv3 run, each under its own time limit.
# usage (GPU box): TAG=r04c bash tools/pmc_cal.sh
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${TAG:-r04c}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="--steps 1 --warmup 0 --no-cpu --no-small-request --no-by-config"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$OUT/${TAG}_wcal_w" -o w --output-format csv -- "$R/tools/wcal" > "$OUT/${TAG}_wcal.txt" &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/${TAG}_wcal_f" -o f --output-format csv -- "$R/tools/wcal" >> "$OUT/${TAG}_wcal.txt" &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex '^k_scan$' -d "$OUT/${TAG}_c4_w" -o w --output-format csv -- python3 "$R/bench.py" $B --config c4 > "$OUT/${TAG}_c4w.json" &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex '^k_scan$' -d "$OUT/${TAG}_c4_f" -o f --output-format csv -- python3 "$R/bench.py" $B --config c4 > "$OUT/${TAG}_c4f.json" &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex '^k_scan$' -d "$OUT/${TAG}_c2_w" -o w --output-format csv -- python3 "$R/bench.py" $B --config c2 > "$OUT/${TAG}_c2w.json" &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex '^k_scan$' -d "$OUT/${TAG}_c2_f" -o f --output-format csv -- python3 "$R/bench.py" $B --config c2 > "$OUT/${TAG}_c2f.json"
