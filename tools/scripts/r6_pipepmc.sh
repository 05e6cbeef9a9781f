#!/bin/bash
# Measurement (GPU box): SQ counters per kernel over the bench's batched pipeline (4 slots x 8
# images, default queues), one rocprofv3 --pmc pass.  Usage: r6_pipepmc.sh TAG STEPS "COUNTERS"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; steps=${2:-8}; CTRS=$3
timeout -s KILL 200 rocprofv3 --pmc $CTRS \
  --output-format csv -d gpurun_out/$tag -o p -- python3 bench.py --batch-only --steps $steps --warmup 2 --no-cpu-baseline --no-pmc \
  > gpurun_out/$tag.log 2>&1 || { tail -5 gpurun_out/$tag.log; exit 1; }
grep '^{' gpurun_out/$tag.log | tail -1 | cut -c1-200
python3 - gpurun_out/$tag <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[k] += 1
names = sorted({c for v in acc.values() for c in v})
print("kernel launches " + " ".join(names))
for k, v in sorted(acc.items(), key=lambda kv: -max(kv[1].values()))[:22]:
    print("  %-36s %5d " % (k[:36], n[k] // len(v)) + " ".join("%14.0f" % v[c] for c in names))
PY
