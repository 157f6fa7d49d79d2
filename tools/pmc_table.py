"""Print kernel-trace averages and per-kernel PMC means of a tools/gpu_pmc_quick.sh run.
    python tools/pmc_table.py TAG [TAG ...]"""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("seb::", "").replace("void ", "")
    return name.split("(")[0][:48]


for tag in sys.argv[1:]:
    d = os.path.join(ROOT, "gpurun_out", f"quick_{tag}")
    print(f"== {tag}")
    for r in csv.DictReader(open(glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))[0])):
        print(f"  {short(r['Name']):50s} calls {r['Calls']:>4s}  avg {float(r['AverageNs']) / 1e3:9.1f} us")
    agg = collections.defaultdict(list)
    for fn in glob.glob(os.path.join(d, "pmc", "*counter_collection.csv")):
        for r in csv.DictReader(open(fn)):
            agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    kern = sorted({k for k, _ in agg})
    ctrs = sorted({c for _, c in agg})
    for k in kern:
        if not k.startswith("k_"):
            continue
        vals = "  ".join(f"{c.replace('SQ_', '')}={sum(agg[(k, c)]) / len(agg[(k, c)]):.3g}" for c in ctrs if (k, c) in agg)
        print(f"  {k:50s} {vals}")
