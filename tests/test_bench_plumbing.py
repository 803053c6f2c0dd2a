"""CPU tests of bench.py's launch plumbing: how --gpus, WORLD_SIZE and the
visible device count decide the mode, the job and the default workload
(VERDICT r01 "make the N>1 bench driver-proof")."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_single_gpu_defaults_to_c4():
    # north_star's scaling job [0, 2^38) at every N, so
    # BENCH's N = 1 line and SCALE's 1/2/4/8 points time the same workload
    r = bench.resolve_run(1, None, {}, visible=1)
    assert r["mode"] == "single" and r["n"] == 1 and r["config"] == "c4"
    assert [c for c, _, _ in bench.SUB_CONFIGS] == ["c2", "c3"]


@pytest.mark.parametrize("n", [2, 4, 8])
def test_library_path_without_torchrun(n):
    # `python bench.py --gpus N` (no WORLD_SIZE): one process, N devices in the library
    r = bench.resolve_run(n, None, {}, visible=8)
    assert r["mode"] == "library" and r["n"] == n and r["world"] == 1
    assert r["config"] == "c4"  # the fixed [0, 2^38) job at N > 1


@pytest.mark.parametrize("n", [2, 8])
def test_torchrun_path(n):
    env = {"WORLD_SIZE": str(n), "RANK": "1", "LOCAL_RANK": "1"}
    r = bench.resolve_run(n, None, env, visible=8)
    assert r["mode"] == "torchrun" and r["n"] == n and r["rank"] == 1 and r["config"] == "c4"


def test_more_gpus_than_visible_is_an_error():
    with pytest.raises(bench.UsageError):
        bench.resolve_run(8, None, {}, visible=1)
    with pytest.raises(bench.UsageError):
        bench.resolve_run(0, None, {}, visible=1)


def test_torchrun_world_mismatch_is_an_error():
    with pytest.raises(bench.UsageError):
        bench.resolve_run(4, None, {"WORLD_SIZE": "2"}, visible=8)


def test_explicit_config_wins():
    assert bench.resolve_run(1, "c4", {}, visible=1)["config"] == "c4"
    assert bench.resolve_run(8, "c2", {}, visible=8)["config"] == "c2"


def test_job_sizes():
    assert bench.job_total(bench.CONFIGS["c4"], 1) == 1 << 38
    assert bench.job_total(bench.CONFIGS["c4"], 8) == 1 << 38  # strong scaling: fixed job
    assert bench.job_total(bench.CONFIGS["c2"], 8) == 8 << 32  # weak scaling
    assert bench.known_answer(bench.CONFIGS["c4"], 8) == bench.known_answer(bench.CONFIGS["c4"], 1)
    assert bench.known_answer(bench.CONFIGS["c2"], 1)[0] == (5256245051, 1626825724)


def test_known_answers_are_independent_pins():
    # every bench workload at N = 1 (and c4 at any N) checks an answer that
    # did not come from the GPU: hashlib (c2) or tools/pin_large.c (c3, c4)
    c2, src2 = bench.known_answer(bench.CONFIGS["c2"], 1)
    c3, src3 = bench.known_answer(bench.CONFIGS["c3"], 1)
    c4, src4 = bench.known_answer(bench.CONFIGS["c4"], 8)
    assert "hashlib" in src2 and "pin_large" in src3 and "pin_large" in src4
    assert c3 == (1902263685, 2962726851) and c4 == (52863133, 182986939864)
    assert bench.known_answer(bench.CONFIGS["c2"], 2) == (None, None)  # [0, 2^33): not pinned


def test_cli_refuses_more_gpus_than_visible():
    # no GPU in this container: --gpus 2 must exit non-zero, never run on fewer
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0
    assert "visible" in p.stderr


def test_host_cores_reports_model():
    n, aff, quota, model = bench.host_cores()
    assert 1 <= n <= aff and model


def test_dist_flag_rehearses_torchrun_path_at_world_one():
    # torchrun --nproc-per-node 1 bench.py --gpus 1 --dist: the RCCL path on one GPU
    r = bench.resolve_run(1, "c4", {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, visible=1, force_dist=True)
    assert r["mode"] == "torchrun" and r["n"] == 1 and r["world"] == 1
    assert bench.resolve_run(1, None, {}, visible=1)["mode"] == "single"  # the driver's N=1 launch


def test_scaling_report_names_the_straggler():
    # 4 GPUs, 10 steps: GPU 2 runs 10% longer kernels, GPU 3 had an empty shard
    units = []
    for i, k in enumerate([1000.0, 1000.0, 1100.0, 0.0]):
        units.append({"rank": i, "shard_lo": 100 * i if k else 1, "shard_hi": 100 * i + 99 if k else 0,
                      "nonces": 10 * (1 << 30) if k else 0, "launches": 10 if k else 0,
                      "alg_ops": 10 * (1 << 30) * 1384 if k else 0, "kernel_ms": k, "scan_ms": k + 5.0,
                      "gather_ms": 0.5})
    rep = bench.scaling_report(units, steps=10, ms_per_step=112.0)
    assert rep["slowest_unit"] == 2
    assert abs(rep["kernel_ms_max_over_mean"] - 110.0 / (310.0 / 3)) < 1e-9
    assert abs(rep["step_ms_not_in_slowest_kernel"] - 2.0) < 1e-9
    assert rep["units"][3]["shard"] is None and rep["units"][3]["frac"] is None
    assert rep["units"][0]["shard"] == [0, 99] and rep["units"][0]["nonces_per_step"] == 1 << 30
    want_frac = (1 << 30) * 1384 / 0.1 / bench.VALU_PEAK_OPS
    assert abs(rep["units"][0]["frac"] - want_frac) < 1e-12
    assert rep["gather_ms_per_step_max"] == 0.05


def _stats(nonces, kernel_ms, b_tail=1, launches=1):
    return {"scan_kernel_ms": kernel_ms, "scan_launches": launches, "scan_nonces": nonces,
            "scan_alg_ops": nonces * 1384 * b_tail, "fast_nonces": nonces, "generic_nonces": 0}


def test_roofline_assembly_c4_fractions_below_one():
    """A realistic c4 run (2^38 nonces in 7.43 s) assembles with every frac
    field <= 1, the one 78.64 T peak, no survey-peak fraction, and the mix
    comparison named as a speed ratio."""
    cfg = bench.CONFIGS["c4"]
    pmc = {"valu_wave_instr_per_nonce": 1186.3, "effective_clock_GHz": 2.384, "hbm_bytes_per_launch": 1.6e6}
    roof = bench.assemble_roofline("c4", cfg, _stats(1 << 38, 7430.0), 1, pmc, "x", (7.427e9, "y"))
    assert abs(roof["peak"] - 78.6432) < 1e-9
    assert 0.6 < roof["frac"] < 0.7 and 0.6 < roof["frac_rocprof"] < 0.7
    assert 0.5 < roof["executed"]["frac"] < 0.6
    assert "frac_vs_survey_peak" not in roof
    mix = roof.get("unhoisted_mix")
    if mix:
        assert "frac" not in mix and mix["speed_vs_unhoisted_mix"] > 1.0


def test_roofline_assembly_round5_c4_dual_issue_fields():
    """The r05t c4 run (2^38 nonces in 5.215 s, PMC VALU2 0.385): frac 0.928,
    the slot-bound mix fraction below 1, and the shared-slot share below its
    bound (a slot pairs any first op with a full-rate second)."""
    cfg = bench.CONFIGS["c4"]
    pmc = {"valu_wave_instr_per_nonce": 1186.3, "effective_clock_GHz": 2.375, "hbm_bytes_per_launch": 1.6e6,
           "dual_valu_issue_quads_per_wave_instr": 0.385}
    roof = bench.assemble_roofline("c4", cfg, _stats(1 << 38, 5215.1), 1, pmc, "x", (5.214e9, "y"))
    assert 0.92 < roof["frac"] < 0.94
    ex = roof["executed"]
    if "mix_issue_frac" in ex:  # needs the committed variant reports
        assert 0.85 < ex["mix_issue_frac"] < 1.0
        d = ex["dual_issue"]
        assert abs(d["valu_ops_in_shared_slots"] - 0.77) < 1e-9
        assert d["valu_ops_in_shared_slots"] <= d["shared_slot_bound"] <= 1.0
        assert abs(d["slot_model_simd_cycles_per_valu"] - 4 * (1 - 0.385)) < 1e-9


def test_roofline_assembly_rejects_work_above_peak():
    """the refusal is on instructions the kernel must
    execute, not on the algorithmic ratio.  The same 2^38 nonces "in" 2 s
    would need the c4 loops' own VALU count at 2x the peak: refused."""
    cfg = bench.CONFIGS["c4"]
    if bench.workload_mix(len(cfg["msg"]), 0, (1 << 38) - 1) is None:
        pytest.skip("variant reports not committed")
    with pytest.raises(bench.RooflineError, match="work_bound"):
        bench.assemble_roofline("c4", cfg, _stats(1 << 38, 2000.0), 1)


def test_sweep_layout_above_one_algorithmically_passes():
    """The r05af sweep's fastest one-block layout (L = 38, d = 16, variant
    [13,6]: 59.79 GH/s, algorithmic frac 1.052; profiles/r05af_layout_sweep.jsonl)
    is a correct run: rounds 0..12 are hoisted, so its loop executes 1035
    VALU per nonce, 0.79 of the peak at that rate.  The line passes with the
    algorithmic ratio above 1 named as a speed ratio."""
    lo = 10 ** 15
    cfg = {"msg": b"m" * 38, "b_tail": 1, "lo": lo, "hi": lo + (1 << 32) - 1}
    assert bench.fast_variant(38, 16) == (13, 6, False)
    ms = (1 << 32) / 59.79169752156909e9 * 1e3
    roof = bench.assemble_roofline("sweep", cfg, _stats(1 << 32, ms), 1)
    assert abs(roof["frac"] - 1.0522) < 1e-3 and "speed ratio" in roof["frac_kind"]
    wb = roof.get("work_bound")
    if wb is not None:  # needs the committed variant reports
        assert wb["loop_valu_per_nonce"] < 1100 and 0.7 < wb["frac"] < 0.9


def test_executed_fraction_above_one_is_refused():
    """A PMC instruction count that this run's rate would execute above the
    peak (executed frac 1.1) means the kernel did not do the work: refused."""
    cfg = bench.CONFIGS["c4"]
    ms = 5188.0
    rate = (1 << 38) / (ms * 1e-3)
    pmc = {"valu_wave_instr_per_nonce": 1.1 * bench.VALU_PEAK_OPS / rate, "effective_clock_GHz": 2.35}
    with pytest.raises(bench.RooflineError, match="executed"):
        bench.assemble_roofline("c4", cfg, _stats(1 << 38, ms), 1, pmc, "x", (5.19e9, "y"), codeobj="h")
    bench.check_work_bound({"frac": 1.3, "frac_rocprof": 1.2, "executed": {"frac": 0.99}})  # algorithmic: allowed
    with pytest.raises(bench.RooflineError):
        bench.check_work_bound({"work_bound": {"frac": 1.01}})


def _decoys(tmp_path, specs):
    """profiles/ with PMC summaries and kernel-trace rows named like real
    sessions: specs = [(tag, config, sha, avg_ns)]"""
    prof = tmp_path / "profiles"
    prof.mkdir()
    for tag, config, sha, avg in specs:
        (prof / f"{tag}_{config}_pmc_summary.json").write_text(
            '{"config": "%s", "codeobj_sha256": "%s", "tag": "%s"}' % (config, sha, tag))
        (prof / f"{tag}_{config}_kernel_stats_workload.csv").write_text(
            '"Name","Calls","AverageNs","Codeobj_SHA256"\n'
            '"k_scan",5,%d,"%s"\n"k_scan (launches after the first 2: timed steps)",3,%d,"%s"\n'
            % (avg + 1, sha, avg, sha))
    return str(tmp_path)


def test_profiles_are_selected_by_code_object_not_name(tmp_path, monkeypatch):
    """r05v sorts after r05ae lexically; the summary of
    the code object the line runs is chosen, the newest session among
    several of it, and a build with no profile gets none."""
    root = _decoys(tmp_path, [("r05v", "c4", "old", 5213000000), ("r05ae", "c4", "new", 5247000000),
                              ("r05z", "c4", "new", 5330000000), ("r05y", "c2", "old", 83760000)])
    monkeypatch.setattr(bench, "ROOT", root)
    assert bench.profile_tag_key("profiles/r05ae_c4_x") > bench.profile_tag_key("profiles/r05z_c4_x") \
        > bench.profile_tag_key("profiles/r05v_c4_x")
    d, src = bench.pmc_summary("c4", "new")
    assert d["tag"] == "r05ae" and src == "profiles/r05ae_c4_pmc_summary.json"
    assert bench.pmc_summary("c4", "old")[0]["tag"] == "r05v"
    assert bench.rocprof_row("c4", "new") == (5247000000.0, "profiles/r05ae_c4_kernel_stats_workload.csv")
    assert bench.pmc_summary("c4", "other") == (None, None) and bench.rocprof_row("c4", "other") == (None, None)
    assert bench.pmc_summary("c2", "new") == (None, None)
    assert bench.pmc_summary("c4", None) == (None, None)


def test_no_profile_of_this_build_leaves_profile_fields_null():
    cfg = bench.CONFIGS["c4"]
    roof = bench.assemble_roofline("c4", cfg, _stats(1 << 38, 5188.0), 1, None, None, (None, None),
                                   codeobj="abc")
    assert roof["profile_stale"] is True and set(roof["profile_missing"]) == {"rocprof", "pmc"}
    assert roof["frac_rocprof"] is None and roof["executed"] is None and roof["traffic"] is None
    assert roof["codeobj_sha256"] == "abc" and 0.9 < roof["frac"] < 0.95


def test_clock_from_stamps_per_xcc():
    """Two probe stamps 100 s apart on a 100 MHz wall counter, XCC x's
    shader counter running at 2.30 + 0.01 x GHz: each XCC's clock, the mean,
    and the XCC's first workgroup as its sample."""
    wall = 100e6
    before, after = [], []
    for b in range(64):
        x = b % 8
        ghz = 2.30 + 0.01 * x
        t, r = 10 ** 9 * (x + 1) + b, 5 * 10 ** 9 + b
        before.append((t, r, t + 40, x))
        r2 = r + int(100 * wall)
        t2 = t + int(100 * ghz * 1e9)
        after.append((t2, r2, t2 + 40, x))
    c = bench.clock_from_stamps(before, after, wall)
    assert abs(c["per_xcc_GHz"]["3"] - 2.33) < 1e-6 and abs(c["mean_GHz"] - 2.335) < 1e-6
    assert abs(c["interval_s"] - 100.0) < 1e-6
    assert bench.clock_from_stamps(before, [], wall) is None


def test_sustained_clock_fraction_in_the_line():
    cfg = bench.CONFIGS["c4"]
    clock = {"effective_clock_GHz": 2.35, "devices": {}}
    roof = bench.assemble_roofline("c4", cfg, _stats(1 << 38, 5188.0), 1, codeobj="h", clock=clock)
    assert roof["effective_clock_GHz"] == 2.35
    assert abs(roof["frac_at_sustained_clock"] - roof["frac"] * 2.4 / 2.35) < 1e-12
    bad = bench.assemble_roofline("c4", cfg, _stats(1 << 38, 5188.0), 1, clock={"effective_clock_GHz": 9.0,
                                                                                "implausible": True})
    assert bad["effective_clock_GHz"] is None and "frac_at_sustained_clock" not in bad


def test_roofline_two_block_config_names_the_algorithmic_ratio():
    cfg = bench.CONFIGS["c3"]
    pmc = {"valu_wave_instr_per_nonce": 893.6, "effective_clock_GHz": 2.375}
    roof = bench.assemble_roofline("c3", cfg, _stats(1 << 34, 343.0, b_tail=2), 1, pmc, "x")
    assert roof["alg_ops_over_peak"] > 1.0  # hoisting + MODE 5: not a utilisation
    assert roof["frac"] is not None and roof["frac"] < 1.0


def test_rocprof_row_reads_committed_summary():
    """The committed c2 trace of the shipped code object (r05ag, retagged
    with its hash) is found by that hash."""
    sha = "ec224f858b5ed8bcd162b07001b8e08ec046635ec5397eaad68df5c39428a78a"
    avg, src = bench.rocprof_row("c2", sha)
    # one c2 launch (2^32 nonces): no faster than the loop's own VALU count
    # allows at the 78.6 T peak, no slower than the round-1 kernel (~120 ms)
    floor = (1 << 32) * 1000 / bench.VALU_PEAK_OPS * 1e9
    assert avg and floor < avg < 130e6 and src.startswith("profiles/"), (avg, src)


def test_bench_refuses_test_knobs():
    """with the master switch set, bench.py exits 4
    before touching a device (no GPU here)."""
    env = dict(os.environ, P1HIP_TEST_KNOBS="1", P1HIP_NO_TABLE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 4, (p.returncode, p.stderr[-2000:])
    assert "P1HIP_NO_TABLE" in p.stderr and "test knobs" in p.stderr


def test_library_ignores_knobs_without_master_switch(monkeypatch):
    import p1_amd

    monkeypatch.setenv("P1HIP_TEST_FAIL_DEVICE", "0")
    monkeypatch.setenv("P1HIP_TEST_KNOBS", "0")
    assert p1_amd.test_knobs() == {}
    monkeypatch.setenv("P1HIP_TEST_KNOBS", "1")
    assert p1_amd.test_knobs() == {"P1HIP_TEST_KNOBS": "1", "P1HIP_TEST_FAIL_DEVICE": "0"}
    monkeypatch.delenv("P1HIP_TEST_KNOBS")
    assert p1_amd.test_knobs() == {}


def test_bench_imports_torch_before_the_library():
    """r04a: loading libp1hip.so before torch leaves two HIP runtimes in the
    process (torch's wheel carries its own) and the second to initialise sees
    no GPU.  main() must import torch before p1_amd."""
    import inspect

    src = inspect.getsource(bench.main)
    assert src.index("import torch\n") < src.index("import p1_amd\n")


SHIPPED_R05 = "ec224f858b5ed8bcd162b07001b8e08ec046635ec5397eaad68df5c39428a78a"


def test_scaling_expectation_for_the_driver_shapes():
    """the N-GPU expectation is this code object's own
    one-GPU c4 rate (its committed trace) x N / the plan_shards balance."""
    for n in (2, 4, 8):
        e = bench.scaling_expectation("c4", n, SHIPPED_R05)
        assert e and e["slowest_shard_over_mean"] < 1.01 and len(e["shard_kernel_ms"]) == n
        assert e["one_gpu_source"].endswith("_c4_kernel_stats_workload.csv") and 51 < e["one_gpu_GH_s"] < 54
        assert abs(e["implied_GH_s"] - n * e["one_gpu_GH_s"] / e["slowest_shard_over_mean"]) < 1e-9
    assert 405 < bench.scaling_expectation("c4", 8, SHIPPED_R05)["implied_GH_s"] < 430
    other = bench.scaling_expectation("c4", 8, "not-profiled")
    assert other["one_gpu_source"] is None and other["implied_GH_s"] > 0
    assert bench.scaling_expectation("c4", 1) is None and bench.scaling_expectation("c2", 8) is None


def test_library_topology_reports_what_rccl_says():
    """a library-mode N-GPU record carries each device's
    communicator size and rank as RCCL reports them (p1hip_comm_info) and a
    world_size taken from them, not a constant."""
    t = bench.library_topology("library", 8, [(8, r) for r in (3, 0, 1, 2, 4, 5, 6, 7)])
    assert t["world_size"] == 8 and t["ranks_in_gather"] == 8 and t["processes"] == 1
    assert t["rccl_ranks"] == [8] * 8 and sorted(t["rccl_rank"]) == list(range(8))
    t1 = bench.library_topology("single", 1, [(0, -1)])
    assert t1["world_size"] == 1 and t1["ranks_in_gather"] is None and t1["rccl_ranks"] == [0]
    assert t1["backend"] is None


@pytest.mark.parametrize("comms", [
    [(1, 0), (1, 0)],            # two one-rank communicators: no cross-GPU gather
    [(2, 0), (2, 0)],            # one rank twice
    [(0, -1), (0, -1)],          # host combine (P1HIP_NO_RCCL)
    [(4, 0), (4, 1)],            # a communicator larger than the run
    [(2, 0)],                    # fewer devices than --gpus
])
def test_library_topology_refuses_a_gather_that_does_not_span_the_gpus(comms):
    with pytest.raises(bench.TopologyError):
        bench.library_topology("library", 2, comms)


def test_bench_exits_5_on_a_bad_communicator():
    """main() queries p1_amd.comm_info after init and exits 5 before timing
    when library_topology refuses."""
    import inspect

    src = inspect.getsource(bench.main)
    assert "comm_info" in src and "sys.exit(5)" in src
    assert src.index("sys.exit(5)") < src.index("timed_steps(")


def test_the_built_code_object_has_committed_profiles():
    """The code object this tree builds has its rocprofv3 trace and PMC
    summaries committed for every BASELINE config the N = 1 line times, so
    the driver's line cites profiles of the kernels it runs (and its
    scaling expectation uses this object's own one-GPU rate)."""
    import p1_amd

    try:
        sha = p1_amd.codeobj_sha256()
    except p1_amd.P1HipError:
        pytest.skip("library not built")
    for config in ("c4", "c2", "c3"):
        pmc, src = bench.pmc_summary(config, sha)
        avg, tsrc = bench.rocprof_row(config, sha)
        assert pmc and avg, (config, sha)
        assert pmc["trace_run"]["avg_launch_ms"] * 1e6 >= avg * 0.999, (config, src, tsrc)
    e = bench.scaling_expectation("c4", 8, sha)
    assert e["one_gpu_source"] == bench.rocprof_row("c4", sha)[1]


def test_layout_config_profiles_one_tail_layout():
    """--layout L,START[,N]: sweep.py's message, one decade, no pinned answer;
    a range that crosses a decade (two kernel variants) is refused."""
    c = bench.layout_config("43,1000000000000000")
    assert c["msg"] == bytes((33 + (i * 7) % 90) for i in range(43)) and c["total"] == 1 << 32
    assert c["layout"] == [43, 16] and c["variant"] == [14, 1, True] and c["b_tail"] == 2
    assert (c["lo"], c["hi"]) == (10**15, 10**15 + (1 << 32) - 1)
    assert bench.known_answer(c, 1) == (None, None)
    assert bench.layout_config("8,1000000000,1000")["b_tail"] == 1
    for bad in ("8", "8,999999999,2", "8,-1", "x,1"):
        with pytest.raises((bench.UsageError, ValueError)):
            bench.layout_config(bad)
