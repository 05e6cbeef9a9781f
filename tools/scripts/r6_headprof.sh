#!/bin/bash
# Measurement (GPU box): kernel stats of the headline pipeline alone (bench.py without the detail
# legs: 4 contexts x batches of 8 synthetic 8192^2 images, encode + decode with the side index),
# then the batch tests (with the batched no-index decode).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6hp -o p -- python3 bench.py --steps 20 --warmup 5 \
  --no-legs --no-pmc --no-cpu-baseline --no-config2 > gpurun_out/r6hp.log 2>&1 || { tail -20 gpurun_out/r6hp.log; exit 1; }
grep '^{' gpurun_out/r6hp.log | tail -1 | cut -c1-160
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r6hp/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:20]:
    print("%-40s calls %6s total %9.2f ms avg %8.3f ms %5.1f%%" % (r["Name"][:40], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
PY
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batch.py 2>&1 | tail -2
