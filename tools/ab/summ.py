"""Summaries of tools/ab runs: fixed-iteration CG timings (ab_pcg.log) and
k_cgs PMC passes (pmc_cgs_*): FETCH_SIZE (x2, gfx950 calibration) / WRITE_SIZE per dispatch."""
import csv
import glob
import json
import os
import statistics
import sys

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
cur = None
for ln in open(os.path.join(out, "ab_pcg.log")):
    if ln.startswith("=="):
        cur = ln.split("/")[-1].strip()
        continue
    try:
        d = json.loads(ln)
    except ValueError:
        continue
    k = d["kernels"]["pcg_iter"]
    print(f"{cur:16s} iters {d['iters']} rel_res {d['rel_res']:.3e} {k['ms_per_launch'] * 1e3:7.2f} us/launch")
for dd in sorted(glob.glob(os.path.join(out, "pmc_cgs_*"))):
    res = {}
    for nm in ("fetch", "write"):
        f = glob.glob(os.path.join(dd, "**", f"{nm}_counter_collection.csv"), recursive=True)
        if not f:
            continue
        vals = {}
        for row in csv.DictReader(open(f[0])):
            if "k_cgs" not in row["Kernel_Name"]:
                continue
            vals.setdefault(row["Dispatch_Id"], 0.0)
            vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
        v = [x for x in vals.values() if x > 0]
        res[nm] = statistics.median(v) / 1e3 if v else None  # KB units -> MB
    print(os.path.basename(dd), json.dumps(res))
