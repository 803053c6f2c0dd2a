#!/bin/bash
# One GPU-box session: VALU micro-benchmark, GPU parity tests, smoke, bench,
# rocprofv3 kernel-trace stats and PMC counter passes.
# Each GPU step has its own time limit.  A test FAILURE (exit 1) does not stop
# the session; any fault/abort/timeout (other non-zero codes) ends it at once.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
TAG=${TAG:-r01}
mkdir -p "$OUT"
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_PEAK:-0}" = 1 ] || step valu_peak 300 "$ROOT/tools/valu_peak" > "$OUT/${TAG}_valu_peak.jsonl"
[ "${RUN_MIX:-0}" != 1 ] || step valu_mix 300 "$ROOT/tools/valu_mix" > "$OUT/${TAG}_valu_mix.jsonl"
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -u -m pytest "$ROOT/tests" -m gpu -x -v -rP -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/${TAG}_pytest_gpu.log" 2>&1
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import sys; sys.path.insert(0, '$ROOT'); import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python "$ROOT/bench.py" ${BENCH_ARGS:-} > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
[ -z "${EXTRA_BENCH:-}" ] || step bench_extra 600 python "$ROOT/bench.py" $EXTRA_BENCH > "$OUT/${TAG}_bench_extra.json" 2> "$OUT/${TAG}_bench_extra.err"
for cfg in ${BENCH_CONFIGS:-}; do
  step bench_$cfg 600 python "$ROOT/bench.py" --config $cfg --steps ${CFG_STEPS:-3} --warmup 1 --no-cpu --no-by-config > "$OUT/${TAG}_bench_$cfg.json" 2> "$OUT/${TAG}_bench_$cfg.err"
done
[ "${RUN_SWEEP:-0}" != 1 ] || step sweep 900 python "$ROOT/tools/sweep.py" > "$OUT/${TAG}_sweep.jsonl" 2> "$OUT/${TAG}_sweep.err"
[ "${RUN_SERVER:-0}" != 1 ] || step bench_server 900 python "$ROOT/tools/bench_server.py" > "$OUT/${TAG}_bench_server.json" 2> "$OUT/${TAG}_bench_server.err"
if [ "${RUN_STRESS:-0}" = 1 ]; then
  # randomized parity against the oracle: production settings, then the
  # fast variants forced onto small ranges (test knobs under their switch)
  step stress 300 python "$ROOT/tools/stress.py" ${STRESS_S:-150} > "$OUT/${TAG}_stress.json" 2> "$OUT/${TAG}_stress.err"
  P1HIP_TEST_KNOBS=1 P1HIP_MIN_FAST_THREADS=1 P1HIP_SMALL_MAX_NONCES=0 step stress_k3 300 python "$ROOT/tools/stress.py" ${STRESS_S:-150} 441 > "$OUT/${TAG}_stress_k3.json" 2> "$OUT/${TAG}_stress_k3.err"
fi
if [ "${RUN_SHARD_BALANCE:-0}" = 1 ]; then
  # the N-GPU plan_shards / equal splits of configs[3], each shard timed alone on GPU 0
  step shard_balance 300 python "$ROOT/tools/shard_balance.py" > "$OUT/${TAG}_shard_balance.jsonl" 2> "$OUT/${TAG}_shard_balance.err"
fi
if [ "${RUN_TORCHRUN8:-0}" = 1 ]; then
  # the driver's N = 8 launch shape on one GPU: 8 ranks, gloo all-gather
  step torchrun8 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 "$ROOT/bench.py" --gpus 8 --steps 2 --warmup 1 --dist-backend gloo > "$OUT/${TAG}_torchrun8.json" 2> "$OUT/${TAG}_torchrun8.err"
fi
if [ "${RUN_TORCHRUN:-0}" = 1 ]; then
  # rehearse the N>1 launch path on one GPU: 2 ranks, gloo all-gather, shared device
  step torchrun2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 "$ROOT/bench.py" --gpus 2 --steps 2 --warmup 1 --dist-backend gloo > "$OUT/${TAG}_torchrun2.json" 2> "$OUT/${TAG}_torchrun2.err"
fi
if [ "${RUN_DIST1:-0}" = 1 ]; then
  # the driver's N>1 code path (torch.distributed "nccl" = RCCL, device_id,
  # all-gather of the 16-B partials, all-reduce of the step time) at world 1
  step dist1_nccl 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 "$ROOT/bench.py" --gpus 1 --dist --config c4 --steps 2 --warmup 1 --no-cpu > "$OUT/${TAG}_dist1_nccl.json" 2> "$OUT/${TAG}_dist1_nccl.err"
fi
# configs[4] end to end over LSP (tools/bench_lsp.py), one run per spec
# "name:VAR=v,VAR=v" (MINERS, COPIES, EPOCH_MS, REPS, HEDGE ...)
for spec in ${LSP_RUNS:-}; do
  name=${spec%%:*}
  vars=${spec#*:}
  step "lsp_$name" 600 env ${vars//,/ } python "$ROOT/tools/bench_lsp.py" > "$OUT/${TAG}_lsp_$name.json" 2> "$OUT/${TAG}_lsp_$name.err"
done
for lib in ${VARIANTS:-}; do
  n=$(basename "$lib" .so)
  P1HIP_LIB="$ROOT/$lib" step "bench_$n" 600 python "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu --no-by-config > "$OUT/${TAG}_bench_$n.json" 2> "$OUT/${TAG}_bench_$n.err"
done
if [ "${RUN_ASAN_TEARDOWN:-0}" = 1 ]; then
  # whose free trips ROCm ASan's "!dev_runtime_unloaded_"
  # at exit.  A HIP + RCCL program without libp1hip (tools/asan_teardown), then
  # the library's stress driver through the normal exit path; every ASan
  # report (stack symbolized) goes to gpurun_out.  Last in the session: an
  # ASan CHECK exits 1, so the steps after it still run.
  step build_sanitize_lib 600 make -s -C "$ROOT" -j16 sanitize-lib
  for m in none malloc rccl; do
    ASAN_OPTIONS="detect_leaks=0:log_path=$OUT/${TAG}_asan_teardown_$m" \
      ASAN_SYMBOLIZER_PATH=/opt/rocm/lib/llvm/bin/llvm-symbolizer \
      step asan_teardown_$m 120 "$ROOT/tools/asan_teardown" $m > "$OUT/${TAG}_asan_teardown_$m.out" 2>&1
  done
  P1_SAN_NORMAL_EXIT=1 ASAN_OPTIONS="detect_leaks=0:log_path=$OUT/${TAG}_san_stress_normal_exit" \
    ASAN_SYMBOLIZER_PATH=/opt/rocm/lib/llvm/bin/llvm-symbolizer \
    step san_stress_normal_exit 240 "$ROOT/tools/san/capi_san_stress" ${SAN_STRESS_S:-20} > "$OUT/${TAG}_san_stress_normal_exit.out" 2>&1
fi
cd /tmp && export TMPDIR=/tmp
# kernel-trace stats and PMC passes of one profiled job (every k_scan launch
# of the profiled command is a workload launch: --no-small-request).  Each
# command's bench JSON line is kept beside its output: it names the code
# object the command ran (library.codeobj_sha256), which
# tools/summarize_prof.py writes into the summaries.
prof_one() {  # prof_one <name> <bench job args...>
  local name=$1; shift
  if [ "${SKIP_PROF:-0}" != 1 ]; then
    # the kernel trace of a bench run shaped like the timed one (warm-up
    # steps, then timed steps): summarize_prof --skip-launches 2 averages the
    # same launches bench.py's own HIP events time
    step rocprof_stats_$name 600 rocprofv3 --kernel-trace --stats -d "$OUT/${TAG}_${name}_prof" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps ${PROF_STEPS:-3} --warmup 2 --no-cpu --no-small-request --no-by-config "$@" > "$OUT/${TAG}_${name}_prof_bench.json"
  fi
  if [ "${SKIP_PMC:-0}" != 1 ]; then
    local i=0 set
    for set in "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VALU_INT32 SQ_INSTS_SALU" \
               "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
               "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH" \
               "FETCH_SIZE" "WRITE_SIZE"; do
      i=$((i+1))
      step pmc_${name}_$i 300 rocprofv3 --pmc $set --kernel-include-regex '^k_scan$' -d "$OUT/${TAG}_${name}_pmc$i" -o pmc --output-format csv -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --no-cpu --no-small-request --no-by-config "$@" > "$OUT/${TAG}_${name}_pmc${i}_bench.json"
    done
  fi
}
for cfg in ${PROF_CONFIGS:-c2}; do
  prof_one "$cfg" --config "$cfg"
done
# one tail layout per spec "L,START[,N]" (bench.py --layout), named L<L>d<digits>
for spec in ${PROF_LAYOUTS:-}; do
  IFS=, read -r L START _ <<< "$spec"
  prof_one "L${L}d${#START}" --layout "$spec"
done
echo "== done"
