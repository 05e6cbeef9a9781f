#!/usr/bin/env python3
"""Per-kernel call count / average / total duration from a rocprofv3 database (rocpd .db) or
kernel_stats.csv.  Usage: kstats.py <dir-or-file> [top]."""
import csv
import glob
import os
import sqlite3
import sys

p = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dbs = [p] if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)
rows = []
if dbs:
    c = sqlite3.connect(dbs[0])
    q = ("select s.kernel_name, count(*), avg(k.end - k.start), sum(k.end - k.start) from rocpd_kernel_dispatch k "
         "join rocpd_info_kernel_symbol s on k.kernel_id = s.id group by s.kernel_name")
    rows = [(n, int(cnt), a / 1e6, t / 1e6) for n, cnt, a, t in c.execute(q)]
else:
    f = glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = [(r["Name"], int(r["Calls"]), float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6)
            for r in csv.DictReader(open(f))]
for n, cnt, a, t in sorted(rows, key=lambda r: -r[3])[:top]:
    print("%-44s %7d %9.4f ms avg %10.2f ms total" % (n[:44], cnt, a, t))
