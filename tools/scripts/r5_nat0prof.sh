#!/bin/bash
# Measurement (GPU box): tools/scripts/nat0_pipe.py under rocprofv3 --kernel-trace: kernel shares.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$tag -o p -- python3 tools/scripts/nat0_pipe.py 4 8 4 \
  > gpurun_out/$tag.log 2>&1 || { tail -5 gpurun_out/$tag.log; exit 1; }
grep '^natural' gpurun_out/$tag.log
python3 - gpurun_out/$tag <<'PY'
import glob, sqlite3, sys
db = sqlite3.connect(glob.glob(sys.argv[1] + "/*.db")[0])
rows = db.execute("select name, count(*), sum(end-start)/1e6 from kernels group by name order by 3 desc").fetchall()
tot = sum(r[2] for r in rows)
for n, c, t in rows[:16]:
    print("  %-40s %5d %10.1f %6.1f%%" % (n[:40], c, t, 100 * t / tot))
PY
