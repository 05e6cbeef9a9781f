#!/bin/bash
# Measurement (GPU box): the bench's batched pipeline alone (4 contexts x batches of 8, HIP's
# default queues) under rocprofv3 --kernel-trace --stats; per-kernel totals per image.
# Usage: bash tools/scripts/r5_pipeprof.sh TAG [STEPS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; steps=${2:-30}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag} -o p -- \
  python3 bench.py --batch-only --steps $steps --warmup 4 --no-cpu-baseline --no-pmc > gpurun_out/${tag}.log 2>&1 \
  || { tail -20 gpurun_out/${tag}.log; exit 1; }
grep '^{' gpurun_out/${tag}.log | tail -1 | cut -c1-400
python3 - gpurun_out/${tag} <<'PY'
import glob, sqlite3, sys
db = sqlite3.connect(glob.glob(sys.argv[1] + "/*.db")[0])
rows = db.execute("select name, count(*), sum(end-start)/1e6 from kernels group by name order by 3 desc").fetchall()
tot = sum(r[2] for r in rows)
print("kernel, launches, total ms, share of kernel time")
for n, c, t in rows[:25]:
    print("  %-44s %6d %10.2f %6.1f%%" % (n[:44], c, t, 100 * t / tot))
PY
