#!/usr/bin/env python3
"""Per-kernel mean of each SQ counter (per dispatch and per wave) from gpu_pmc_sq.sh output dirs."""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(f"{sys.argv[1]}/*/*/*counter_collection.csv") +
                   glob.glob(f"{sys.argv[1]}/*/*counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lbk::", "")
        if "lbk" not in r["Kernel_Name"]:
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    waves = sum(cs["SQ_WAVES"]) / max(1, len(cs["SQ_WAVES"])) if "SQ_WAVES" in cs else None
    print(f"## {k}  (waves/dispatch {waves})")
    for c, v in sorted(cs.items()):
        m = sum(v) / len(v)
        per = f"{m / waves:12.1f}/wave" if waves else ""
        print(f"  {c:24s} {m:16.1f} {per}")
