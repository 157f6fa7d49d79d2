"""Per-variant kernel averages of a tools/gpu_prof_variants.sh run: python tools/pv_table.py TAG"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"pv_{sys.argv[1]}", "*"))):
    line = next((x for x in open(os.path.join(d, "log")) if x.startswith("{")), None)
    head = ""
    if line:
        j = json.loads(line)
        head = f"build {j.get('build_ms')} probe {j.get('probe_ms')} value {j['value']}"
    print(f"== {os.path.basename(d)}  {head}")
    for f in glob.glob(os.path.join(d, "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if "seb::" in r["Name"]:
                name = re.sub(r"\(.*", "", r["Name"].replace("void ", "").replace("seb::", ""))
                print(f"   {name[:60]:60s} {r['Calls']:>4s} {float(r['AverageNs']) / 1e3:8.1f} us")
