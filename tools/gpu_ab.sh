#!/bin/bash
# A/B of alternative library builds on the MI355X: per library, a c2 and a
# c4 bench (kernel rate from HIP events) and one PMC pass over c2 for the
# dual-issue share (SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU).  The shipped
# library runs first and last (drift control).
# usage: TAG=r05f LIBS="p1_amd/variants/libp1hip_x.so ..." tools/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-r05}
mkdir -p "$OUT"
C2STEPS=${C2STEPS:-10}
C4STEPS=${C4STEPS:-2}
run() {  # run <name> <lib>
  local name=$1 lib=$2
  echo "== $name ($(date +%T))"
  P1HIP_LIB="$lib" timeout -k 10 300 python "$ROOT/bench.py" --config c2 --steps $C2STEPS --warmup 2 --no-cpu --no-by-config --no-small-request > "$OUT/${TAG}_${name}_c2.json" 2> "$OUT/${TAG}_${name}_c2.err" || return $?
  if [ "${C3STEPS:-0}" != 0 ]; then
    P1HIP_LIB="$lib" timeout -k 10 300 python "$ROOT/bench.py" --config c3 --steps $C3STEPS --warmup 1 --no-cpu --no-by-config --no-small-request > "$OUT/${TAG}_${name}_c3.json" 2> "$OUT/${TAG}_${name}_c3.err" || return $?
  fi
  if [ "$C4STEPS" != 0 ]; then
    P1HIP_LIB="$lib" timeout -k 10 300 python "$ROOT/bench.py" --config c4 --steps $C4STEPS --warmup 1 --no-cpu --no-by-config --no-small-request > "$OUT/${TAG}_${name}_c4.json" 2> "$OUT/${TAG}_${name}_c4.err" || return $?
  fi
  (cd /tmp && P1HIP_LIB="$lib" TMPDIR=/tmp timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE SQ_WAVES --kernel-include-regex '^k_scan$' -d "$OUT/${TAG}_${name}_pmc" -o pmc --output-format csv -- python3 "$ROOT/bench.py" --config c2 --steps 1 --warmup 0 --no-cpu --no-by-config --no-small-request > /dev/null) || return $?
}
run base "$ROOT/p1_amd/libp1hip.so" || exit $?
for lib in $LIBS; do
  n=$(basename "$lib" .so); n=${n#libp1hip_}
  run "$n" "$ROOT/$lib" || exit $?
done
run base2 "$ROOT/p1_amd/libp1hip.so" || exit $?
echo "== ab done"
