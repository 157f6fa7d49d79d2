"""Print the MultiGet kernels' average durations (us) of a tools/mg_ab.sh run.
    python tools/mg_ab_stats.py TAG"""
import csv
import glob
import json
import os
import sys

for d in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/*/")):
    for c in ("lsm", "lsm_wide"):
        f = os.path.join(d, c, "k_kernel_stats.csv")
        if not os.path.exists(f):
            continue
        ks = {r["Name"].split("(")[0].replace("void ", "").replace("seb::", "")[:20]: float(r["AverageNs"]) / 1e3
              for r in csv.DictReader(open(f)) if "mg" in r["Name"] or "multiget" in r["Name"]}
        try:
            line = json.loads(open(os.path.join(d, c + ".json")).read().strip().splitlines()[-1])
            ms = line["ms_per_step"]
        except Exception:
            ms = None
        print(os.path.basename(d.rstrip("/")), c, ms, {k: round(v, 1) for k, v in ks.items()})
