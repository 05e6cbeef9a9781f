#!/bin/bash
# Measurement (GPU box): kernel stats of the natural -s0 pipeline (nat0_pipe.py: 4 contexts x
# batches of 8 natural 8192^2 images, encode + decode with the side index).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/scripts/nat0_pipe.py 4 8 10 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6n0 -o p -- python3 tools/scripts/nat0_pipe.py 4 8 10 \
  > gpurun_out/r6n0.log 2>&1 || { tail -20 gpurun_out/r6n0.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r6n0/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:18]:
    print("%-40s calls %6s total %9.2f ms avg %8.3f ms %5.1f%%" % (r["Name"][:40], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
PY
