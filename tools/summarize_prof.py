"""Copy one GPU session's rocprofv3 outputs from gpurun_out/ into profiles/
and write a JSON summary of the scan kernel's counters.

usage: python tools/summarize_prof.py <TAG> [nonces_per_launch] [--config cN --nonces-total N]
  reads  gpurun_out/<TAG>_prof/run_kernel_stats.csv  (--kernel-trace --stats)
         gpurun_out/<TAG>_pmc*/pmc_counter_collection.csv (--pmc passes)
         gpurun_out/<TAG>_bench*.json, <TAG>_valu_*.jsonl
  writes profiles/<TAG>_kernel_stats.csv, profiles/<TAG>_pmc_summary.json,
         profiles/<TAG>_bench*.json, profiles/<TAG>_valu_*.jsonl
  With --nonces-total (the nonces the profiled command scanned, every k_scan
  launch of it a workload launch: bench.py --no-small-request), per-nonce
  figures come from counters summed over ALL its launches -- needed when a
  step is several launches (configs[3]: 2 per 2^38 scan).

  Every summary names the code object it measured:
  `codeobj_sha256` in the PMC summary and a Codeobj_SHA256 column in the
  workload CSV, read from the JSON lines the profiled bench commands printed
  (gpurun_out/<TAG>_prof_bench.json, <TAG>_pmc*_bench.json: bench.py's
  library.codeobj_sha256).  The commands must agree; bench.py cites only
  summaries whose hash equals the code object it runs.

  python tools/summarize_prof.py --retag TAG --codeobj-sha256 H --basis TEXT
  adds the hash to an already committed TAG's summaries (profiles taken
  before the hash was recorded), with the basis for the attribution.
"""
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def codeobj_of(src, tag, explicit=None):
    """sha256 of the code object the profiled commands of `tag` ran: every
    bench JSON line they printed must name the same one (and match
    `explicit` when given).  Raises SystemExit otherwise."""
    seen = {}
    for f in sorted(glob.glob(os.path.join(src, f"{tag}_prof_bench.json")) +
                    glob.glob(os.path.join(src, f"{tag}_pmc*_bench.json"))):
        for ln in open(f):
            if ln.startswith("{"):
                h = json.loads(ln).get("library", {}).get("codeobj_sha256")
                if h:
                    seen[os.path.basename(f)] = h
    got = set(seen.values())
    if explicit:
        if got - {explicit}:
            raise SystemExit(f"summarize_prof: --codeobj-sha256 {explicit} but the profiled commands ran {seen}")
        return explicit, "given" if not seen else sorted(seen)
    if len(got) != 1:
        raise SystemExit(f"summarize_prof: need exactly one code object across the profiled commands, got {seen} "
                         f"(pass --codeobj-sha256 for output without bench lines)")
    return got.pop(), sorted(seen)


def trace_run(src, tag):
    """What the kernel-trace command's own bench line measured (its timed
    steps, the shader clock its probe read): the trace's launch time and
    the clock it ran at, side by side."""
    f = os.path.join(src, f"{tag}_prof_bench.json")
    if not os.path.exists(f):
        return None
    for ln in open(f):
        if ln.startswith("{"):
            d = json.loads(ln)
            r = d.get("roofline", {})
            return {"ms_per_step": d.get("ms_per_step"), "avg_launch_ms": r.get("avg_launch_ms"),
                    "effective_clock_GHz": r.get("effective_clock_GHz"), "steps": d.get("steps"),
                    "source": os.path.basename(f)}
    return None


def retag(tag, sha, basis):
    """Add the code object hash to an already committed TAG's summaries."""
    dst = os.path.join(ROOT, "profiles")
    done = []
    p = os.path.join(dst, f"{tag}_pmc_summary.json")
    if os.path.exists(p):
        d = json.load(open(p))
        d["codeobj_sha256"], d["codeobj_source"] = sha, {"retagged": basis}
        with open(p, "w") as f:
            json.dump(d, f, indent=1)
        done.append(p)
    p = os.path.join(dst, f"{tag}_kernel_stats_workload.csv")
    if os.path.exists(p):
        rows = list(csv.DictReader(open(p)))
        def num(v):
            for t in (int, float):
                try:
                    return t(v)
                except ValueError:
                    pass
            return v
        write_stats_rows(p, [dict({k: num(v) for k, v in r.items()}, Codeobj_SHA256=sha) for r in rows])
        done.append(p)
    if not done:
        raise SystemExit(f"summarize_prof: nothing committed under profiles/ for {tag}")
    return done


STATS_COLS = ["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "StdDev", "Grid_Size_X", "Source",
              "Codeobj_SHA256"]


def write_stats_rows(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=STATS_COLS, quoting=csv.QUOTE_NONNUMERIC, extrasaction="ignore")
        w.writeheader()
        for r in rows:
            w.writerow({k: r.get(k, "") for k in STATS_COLS})


def workload_stats(trace, out, skip=0, codeobj=""):
    """rocprofv3 --kernel-trace rows of the workload's k_scan launches only
    (largest grid; bench.py's configs[0]-sized latency probe launches small
    grids of the same kernel), in the --stats CSV layout.  With skip > 0 a
    second row covers the launches after the first `skip` (the profiled
    bench command's warm-up steps), i.e. the same launches bench.py's own
    HIP events time."""
    rows = [r for r in csv.DictReader(open(trace)) if r["Kernel_Name"].split("(")[0] == "k_scan"]
    if not rows:
        return
    g = max(int(r["Grid_Size_X"]) for r in rows)
    rows = sorted((r for r in rows if int(r["Grid_Size_X"]) == g), key=lambda r: int(r["Start_Timestamp"]))
    d_all = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
    out_rows = []
    for name, d in (("k_scan", d_all), (f"k_scan (launches after the first {skip}: timed steps)", d_all[skip:])):
        if not d or (name != "k_scan" and skip == 0):
            continue
        mean = sum(d) / len(d)
        sd = (sum((x - mean) ** 2 for x in d) / len(d)) ** 0.5
        out_rows.append({"Name": name, "Calls": len(d), "TotalDurationNs": sum(d), "AverageNs": round(mean, 1),
                         "MinNs": min(d), "MaxNs": max(d), "StdDev": round(sd, 1), "Grid_Size_X": g,
                         "Source": os.path.basename(trace), "Codeobj_SHA256": codeobj})
    write_stats_rows(out, out_rows)


# Measured issue cost (SIMD cycles per wave instruction at 4 waves/SIMD,
# 8-byte encodings at 4 mod 8: DESIGN.md 4 "What bounds it") of the two
# integer-VALU classes; used to price an executed mix.
ISSUE_COST_HALF = 4.37   # v_alignbit_b32, v_add3_u32 and the other 3-input VOP3 ops
ISSUE_COST_FULL = 2.66   # v_bitop3_b32, v_add_u32_e64, v_lshrrev_b32_e64, ...


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--codeobj-sha256", default=None)
    ap.add_argument("--retag", action="store_true", help="add --codeobj-sha256 to TAG's committed summaries")
    ap.add_argument("--basis", default=None, help="--retag: why the profile is of that code object")
    ap.add_argument("nonces_per_launch", nargs="?", type=float, default=2.0**32)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--nonces-total", type=float, default=None)
    ap.add_argument("--skip-launches", type=int, default=0,
                    help="warm-up launches of the profiled command (second row of the workload stats)")
    ap.add_argument("--tiles", type=int, default=None,
                    help="k_scan tiles (16-B partials) per launch: since round 6 the grid is the device's "
                         "workgroup slots and not the tiles (work queue), so the partial bytes need the count")
    ap.add_argument("--half-rate-share", type=float, default=None,
                    help="share of class-A (half-rate) instructions in the executed loop mix")
    a = ap.parse_args()
    tag, nonces = a.tag, a.nonces_per_launch
    if a.retag:
        if not (a.codeobj_sha256 and a.basis):
            raise SystemExit("summarize_prof: --retag needs --codeobj-sha256 and --basis")
        print("\n".join(retag(tag, a.codeobj_sha256, a.basis)))
        return
    src = os.path.join(ROOT, "gpurun_out")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    codeobj, codeobj_src = codeobj_of(src, tag, a.codeobj_sha256)
    ks = os.path.join(src, f"{tag}_prof", "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    kt = os.path.join(src, f"{tag}_prof", "run_kernel_trace.csv")
    if os.path.exists(kt):
        workload_stats(kt, os.path.join(dst, f"{tag}_kernel_stats_workload.csv"), a.skip_launches, codeobj)
    for f in (glob.glob(os.path.join(src, f"{tag}_bench*.json")) + glob.glob(os.path.join(src, f"{tag}_valu_*.jsonl"))
              + glob.glob(os.path.join(src, f"{tag}_prof_bench.json"))):
        shutil.copy(f, os.path.join(dst, os.path.basename(f)))
    counters, durs, sums = {}, [], {}
    gmax_all = 0  # largest k_scan grid (threads) seen in the PMC passes
    for f in sorted(glob.glob(os.path.join(src, f"{tag}_pmc*", "*counter_collection.csv"))):
        rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].split("(")[0] == "k_scan"]
        if not rows:
            continue
        # only the workload's own launches (largest grid); bench.py also times
        # small configs[0]-sized requests whose launches are not the roofline kernel
        gmax = max(int(r["Grid_Size"]) for r in rows)
        gmax_all = max(gmax_all, gmax)
        for r in rows:
            sums[r["Counter_Name"]] = sums.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if int(r["Grid_Size"]) != gmax:
                continue
            counters.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    if not counters:
        print("no PMC data for", tag)
        return
    avg = {k: sum(v) / len(v) for k, v in counters.items()}
    dur = sum(durs) / len(durs)
    out = {"tag": tag, "config": a.config, "kernel": "k_scan", "avg_duration_s": dur,
           "counters_per_launch": avg, "codeobj_sha256": codeobj, "codeobj_source": codeobj_src}
    tr = trace_run(src, tag)
    if tr:
        out["trace_run"] = tr
    if a.nonces_total:
        out["nonces_total"] = a.nonces_total
        out["counters_total"] = sums
    if "GRBM_GUI_ACTIVE" in avg:
        out["effective_clock_GHz"] = avg["GRBM_GUI_ACTIVE"] / 8 / dur / 1e9  # summed over 8 XCDs
    if "SQ_INSTS_VALU" in avg:
        if a.nonces_total:
            out["valu_wave_instr_per_nonce"] = sums["SQ_INSTS_VALU"] * 64 / a.nonces_total
        else:
            out["valu_wave_instr_per_nonce"] = avg["SQ_INSTS_VALU"] * 64 / nonces
        if "effective_clock_GHz" in out:
            simd_cycles = dur * out["effective_clock_GHz"] * 1e9 * 1024
            out["simd_cycles_per_valu_wave_instr"] = simd_cycles / avg["SQ_INSTS_VALU"]
            out["valu_issue_frac_of_2cyc_peak"] = 2.0 / out["simd_cycles_per_valu_wave_instr"]
            if a.half_rate_share is not None:
                # executed mix priced at the measured class issue costs / SIMD cycles spent
                price = a.half_rate_share * ISSUE_COST_HALF + (1 - a.half_rate_share) * ISSUE_COST_FULL
                out["half_rate_share"] = a.half_rate_share
                out["issue_frac"] = price / out["simd_cycles_per_valu_wave_instr"]
    if "SQ_ACTIVE_INST_VALU" in avg and "GRBM_GUI_ACTIVE" in avg:
        # VALUBusy's own expression (rocprofv3 --list-avail): quad-cycles of
        # VALU work per CU over GPU cycles (GRBM_GUI_ACTIVE is summed over 8 XCDs)
        gpu_cycles = avg["GRBM_GUI_ACTIVE"] / 8
        out["valu_busy_frac"] = avg["SQ_ACTIVE_INST_VALU"] * 4 / 256 / gpu_cycles / 4
        out["valu_busy_note"] = ("SQ_ACTIVE_INST_VALU x 4 cycles / (256 CUs x 4 SIMDs x GPU cycles); "
                                 "on gfx950 this counter equals SQ_INSTS_VALU (one count per wave "
                                 "instruction), so it measures issue slots, not busy cycles")
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_INSTS_VALU" in avg:
        out["thread_cycles_valu_per_wave_instr"] = avg["SQ_THREAD_CYCLES_VALU"] / avg["SQ_INSTS_VALU"]
    if "SQ_ACTIVE_INST_VALU2" in avg and "SQ_INSTS_VALU" in avg:
        out["dual_valu_issue_quads_per_wave_instr"] = avg["SQ_ACTIVE_INST_VALU2"] / avg["SQ_INSTS_VALU"]
    if "SQ_BUSY_CU_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        out["cu_busy_frac"] = avg["SQ_BUSY_CU_CYCLES"] * 4 / 256 / (avg["GRBM_GUI_ACTIVE"] / 8)
    if "FETCH_SIZE" in avg or "WRITE_SIZE" in avg:
        # FETCH_SIZE/WRITE_SIZE are KB; gfx950 FETCH_SIZE under-counts wide streaming reads 2x
        # (MI355X_MICROARCH.md HBM section) -- this kernel has no such reads (kernel args,
        # a <4 KB segment table via scalar loads, 16-B partial stores), so no correction applies.
        out["hbm_bytes_per_launch"] = (avg.get("FETCH_SIZE", 0.0) + avg.get("WRITE_SIZE", 0.0)) * 1024
        out["fetch_bytes_per_launch"] = avg.get("FETCH_SIZE", 0.0) * 1024
        out["write_bytes_per_launch"] = avg.get("WRITE_SIZE", 0.0) * 1024
        # k_scan stores one 16-B partial per 256-thread workgroup; the
        # calibration kernel of the same pattern (tools/wcal.hip) gives the
        # factor WRITE_SIZE counts it with (profiles/*_wcal.json)
        cal = sorted(glob.glob(os.path.join(dst, "*_wcal.json")))
        if cal and "WRITE_SIZE" in avg:
            c = json.load(open(cal[-1]))
            factor = c["k_part16"]["counted_over_actual"]
            out["write_bytes_per_launch_calibrated"] = out["write_bytes_per_launch"] / factor
            tiles = a.tiles if a.tiles else gmax_all / 256  # static grid (round 5 and before): workgroups = tiles
            out["partials_bytes_per_launch"] = tiles * 16
            out["tiles_per_launch"] = tiles
            out["traffic_note"] = (f"raw FETCH_SIZE+WRITE_SIZE per k_scan launch; WRITE_SIZE counts k_scan's "
                                   f"16-B-per-workgroup partial stores {factor:.2f}x "
                                   f"({os.path.relpath(cal[-1], ROOT)}), so the calibrated write bytes are "
                                   f"write_bytes_per_launch_calibrated against partials_bytes_per_launch "
                                   f"(16 B x tiles); FETCH is kernel arguments and segment tables; since round 6 "
                                   f"the work queue adds one agent-scope atomic per tile (and one per workgroup "
                                   f"at exit), which the write counters see as well")
    with open(os.path.join(dst, f"{tag}_pmc_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
