#!/usr/bin/env python3
"""Kernel timeline of the last encode in a rocprofv3 (rocpd) database: name, duration, start, end
relative to the encode's first kernel (FIRST, default k_front256).
    python3 tools/scripts/timeline.py DB [FIRST] [MIN_MS]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
first = sys.argv[2] if len(sys.argv) > 2 else "k_front256"
mn = float(sys.argv[3]) if len(sys.argv) > 3 else 0.2
rows = db.execute("select name, (end-start)/1e6, start, end from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if r[0].startswith(first)][-1]
t0 = rows[idx][2]
for n, d, s, e in rows[idx:]:
    if d > mn:
        print("  %-34s %8.3f  %8.3f -> %8.3f" % (n[:34], d, (s - t0) / 1e6, (e - t0) / 1e6))
