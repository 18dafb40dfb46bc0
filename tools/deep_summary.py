"""Summarise tools/deep_profile.sh output per kernel (sums over launches) and drop the raw CSVs.
usage: python tools/deep_summary.py OUTDIR > OUTDIR/summary.json"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

out = sys.argv[1]
res = defaultdict(lambda: defaultdict(float))
calls = defaultdict(int)
for d in sorted(glob.glob(os.path.join(out, "*/"))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
            res[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if os.path.basename(d.rstrip("/")) == "sq2" and r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                calls[k] += 1
    shutil.rmtree(d)
print(json.dumps({k: dict(v, calls=calls.get(k, 0)) for k, v in res.items() if k.startswith("k_")}, indent=1))
