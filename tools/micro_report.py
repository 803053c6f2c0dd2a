"""Join an issue-rate microbenchmark's timing lines (tools/dual or
tools/loopbench, run by tools/gpu_micro.sh) with its PMC pass: per kernel,
SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU (the share of VALU instructions issued
two to a quad-cycle) and the slot model's prediction
4 x (1 - VALU2/VALU) SIMD cycles per VALU instruction beside the measured
one.  Writes profiles/<TAG>_<BIN>_report.jsonl.

usage: micro_report.py TAG BIN      (e.g. r05d loopbench)"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, binname = sys.argv[1], sys.argv[2]
    out_dir = os.path.join(ROOT, "gpurun_out")
    timing = [json.loads(ln) for ln in open(os.path.join(out_dir, f"{tag}_{binname}.jsonl")) if ln.startswith("{")]
    # kernel name -> (label fields) from the generated source's run() calls
    order = []
    for ln in open(os.path.join(ROOT, "tools", f"{binname}.hip")):
        m = re.search(r"run\((k\d+), \"([^\"]+)\", (\d+)", ln)
        if m:
            order.append((m.group(1), m.group(2), int(m.group(3))))
    label = {k: (n, a) for k, n, a in order}
    pmc = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(out_dir, f"{tag}_{binname}pmc", "pmc_counter_collection.csv"))):
        k = r["Kernel_Name"].split("(")[0]
        if k not in label:
            continue
        key = (k, int(r["Grid_Size"]) // 256 // 256)  # waves per SIMD on 256 CUs
        pmc[key][r["Counter_Name"]] = pmc[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    rows = []
    for t in timing:
        if "device" in t:
            continue
        name = t.get("pattern", t.get("variant"))
        wps = t.get("waves_per_simd", 4)
        k = next(k for k, (n, a) in label.items() if n == name and a == t["align"])
        c = pmc.get((k, wps), {})
        frac2 = c.get("SQ_ACTIVE_INST_VALU2", 0.0) / c["SQ_INSTS_VALU"] if c.get("SQ_INSTS_VALU") else None
        row = dict(t)
        row["valu2_per_valu"] = frac2
        if frac2 is not None and wps > 1:
            row["slot_model_cyc_per_valu"] = 4.0 * (1.0 - frac2)
        if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_INSTS_VALU"):
            # GPU-busy cycles (GRBM_GUI_ACTIVE is summed over the 8 XCDs) x
            # 1024 SIMDs per VALU wave-instruction: the whole dispatch,
            # ramp-up and drain included
            row["gui_cyc_per_valu"] = c["GRBM_GUI_ACTIVE"] / 8 * 1024 / c["SQ_INSTS_VALU"]
        rows.append(row)
    dst = os.path.join(ROOT, "profiles", f"{tag}_{binname}_report.jsonl")
    with open(dst, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    print(dst)


if __name__ == "__main__":
    main()
