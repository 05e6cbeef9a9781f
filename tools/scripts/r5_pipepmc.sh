#!/bin/bash
# Measurement (GPU box): instruction mix per kernel over the bench's batched pipeline (4 slots x 8
# images, default queues), one rocprofv3 --pmc pass of SQ counters.  Usage: r5_pipepmc.sh TAG STEPS
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; steps=${2:-8}
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
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
    if r["Counter_Name"] == "SQ_WAVES": n[k] += 1
print("kernel, launches, VALU, SALU, LDS, VMEM rd, VMEM wr (wave-instructions, all launches), waves, wave-cycles")
tot = sum(v["SQ_INSTS_VALU"] for v in acc.values())
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]["SQ_INSTS_VALU"])[:20]:
    print("  %-36s %5d %14.0f %12.0f %12.0f %12.0f %12.0f %10.0f %14.0f  (%.1f%% of VALU)" % (
        k[:36], n[k], v["SQ_INSTS_VALU"], v["SQ_INSTS_SALU"], v["SQ_INSTS_LDS"], v["SQ_INSTS_VMEM_RD"], v["SQ_INSTS_VMEM_WR"],
        v["SQ_WAVES"], v["SQ_WAVE_CYCLES"], 100 * v["SQ_INSTS_VALU"] / tot))
PY
