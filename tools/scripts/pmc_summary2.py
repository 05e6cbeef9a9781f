#!/usr/bin/env python3
"""Per-kernel average of every counter in one or more rocprofv3 --pmc counter_collection.csv
trees: pmc_summary2.py DIR [DIR...] [--kernels k1,k2].  Prints one line per kernel."""
import csv
import glob
import os
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
want = None
for a in sys.argv[1:]:
    if a.startswith("--kernels="):
        want = a.split("=", 1)[1].split(",")
acc = {}
for d in args:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].strip()
            if want and k not in want:
                continue
            e = acc.setdefault(k, {})
            c = e.setdefault(row["Counter_Name"], [0.0, set()])
            c[0] += float(row["Counter_Value"])
            c[1].add(row["Dispatch_Id"])
for k in sorted(acc):
    print(k, " ".join("%s=%.4g" % (c, v[0] / len(v[1])) for c, v in sorted(acc[k].items())))
