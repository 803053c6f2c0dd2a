"""Summarise a tools/gpu_ab.sh session: per library build, the c2 / c4
kernel rates of bench.py and, from the c2 PMC pass, VALU instructions per
nonce, the dual-issue share (SQ_ACTIVE_INST_VALU2 / SQ_INSTS_VALU) and SIMD
cycles per VALU instruction.  Writes profiles/<TAG>_ab.jsonl.

usage: ab_report.py TAG"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_line(path):
    if not os.path.exists(path):
        return None
    for ln in open(path):
        if ln.startswith("{"):
            return json.loads(ln)
    return None


def main():
    tag = sys.argv[1]
    out_dir = os.path.join(ROOT, "gpurun_out")
    names = []
    for p in sorted(glob.glob(os.path.join(out_dir, f"{tag}_*_c2.json")), key=os.path.getmtime):
        names.append(os.path.basename(p)[len(tag) + 1:-len("_c2.json")])
    rows = []
    for n in names:
        r = {"build": n}
        for cfg in ("c2", "c3", "c4"):
            b = bench_line(os.path.join(out_dir, f"{tag}_{n}_{cfg}.json"))
            if b:
                r[cfg] = {"GH_s": b["value"], "frac": b["roofline"].get("frac"),
                          "kernel_GH_s": b["roofline"].get("kernel_hashes_per_s_G"), "avg_launch_ms": b["roofline"].get("avg_launch_ms"),
                          "matches_known": b["result"]["matches_known"]}
        pmc = glob.glob(os.path.join(out_dir, f"{tag}_{n}_pmc", "pmc_counter_collection.csv"))
        if pmc:
            c = {}
            for x in csv.DictReader(open(pmc[0])):
                c[x["Counter_Name"]] = c.get(x["Counter_Name"], 0.0) + float(x["Counter_Value"])
            nonces = 2 ** 32
            r["c2_pmc"] = {"valu_per_nonce": c["SQ_INSTS_VALU"] * 64 / nonces,
                           "valu2_per_valu": c["SQ_ACTIVE_INST_VALU2"] / c["SQ_INSTS_VALU"],
                           "simd_cyc_per_valu": c["GRBM_GUI_ACTIVE"] / 8 * 1024 / c["SQ_INSTS_VALU"]}
        rows.append(r)
    dst = os.path.join(ROOT, "profiles", f"{tag}_ab.jsonl")
    with open(dst, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
            print(json.dumps(r))


if __name__ == "__main__":
    main()
