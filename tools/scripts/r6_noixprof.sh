#!/bin/bash
# Measurement (GPU box): kernel stats of the no-index pipeline (bench.py --no-index, 4 contexts x
# batches of 8) under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6nx -o p -- python3 bench.py --no-index --steps 10 --warmup 3 \
  --no-legs --no-pmc --no-cpu-baseline --no-config2 > gpurun_out/r6nx.log 2>&1 || { tail -20 gpurun_out/r6nx.log; exit 1; }
grep '^{' gpurun_out/r6nx.log | tail -1 | cut -c1-200
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r6nx/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print("%-40s calls %6s total %9.2f ms avg %8.3f ms %5.1f%%" % (r["Name"][:40], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
PY
