#!/bin/bash
# Measurement (GPU box): HBM traffic per launch of the -sN encode kernels on the natural 8192^2
# image -- two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE: they do not fit one pass), gfx950
# correction hbm = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md), per kernel the mean over
# its launches.  Usage: bash tools/scripts/r5_spmc.sh TAG SPEED
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; sp=$2
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/${tag}_$ctr -o p -- \
    python3 tools/scripts/natural_prof.py 8192 $sp 2 > gpurun_out/${tag}_$ctr.log 2>&1 || { tail -5 gpurun_out/${tag}_$ctr.log; exit 1; }
done
python3 - gpurun_out/${tag} <<'PY'
import csv, glob, sys, collections
base = sys.argv[1]
vals = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(base + "_" + ctr + "/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    vals[ctr] = {k: sum(v) / len(v) for k, v in acc.items()}
print("kernel, FETCH_SIZE KB, WRITE_SIZE KB, hbm MB per launch (2 x fetch + write)")
rows = []
for k in vals["FETCH_SIZE"]:
    fe, wr = vals["FETCH_SIZE"][k], vals["WRITE_SIZE"].get(k, 0.0)
    rows.append((2 * fe * 1024 + wr * 1024, k, fe, wr))
for hb, k, fe, wr in sorted(rows, reverse=True)[:20]:
    print("  %-32s %12.0f %12.0f %10.1f" % (k[:32], fe, wr, hb / 1e6))
PY
