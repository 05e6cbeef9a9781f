#!/bin/bash
# Measurement (GPU box): k_lzsort's grid (knob LZSORT_GRID: tiles strided over fewer workgroups)
# and workgroup size (a library built with -DLZSORT_T=...) against its time, the search kernels
# beside it, its fabric traffic and the natural 8192^2 -s1 / -s4 encodes.  LIB: a knobs build
# (tools/scripts/mkknobs.sh / mkvariant.sh).  Usage: r5_lzsortgrid.sh TAG "GRIDS" LIB
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; grids=${2:-"0 512 256 128 64"}; lib=${3:-var/knobs.so}
for g in $grids; do
  for sp in 1 4; do
    d=gpurun_out/${tag}_g${g}_s$sp
    HOH_LIB=$lib HOH_LZSORT_GRID=$g timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o p -- \
      python3 tools/scripts/natural_prof.py 8192 $sp 3 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    python3 - $d "grid $g -s$sp: $(grep '^natural' $d.log | sed 's/.*B (sha/(sha/;s/, decode.*//')" <<'PY'
import glob, sqlite3, sys
db = sqlite3.connect(glob.glob(sys.argv[1] + "/*.db")[0])
out = []
for k in ("k_lzsort", "k_lzscreen", "k_lzscan", "k_search_walk_multi", "k_search(", "k_lzvert"):
    r = db.execute("select avg(end-start)/1e6 from kernels where name like ?", (k + "%",)).fetchone()
    out.append("%s %.2f" % (k.rstrip("("), r[0] or 0))
print(sys.argv[2] + " | " + ", ".join(out))
PY
  done
  d=gpurun_out/${tag}_g${g}_pmc
  HOH_LIB=$lib HOH_LZSORT_GRID=$g timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d -o p -- \
    python3 tools/scripts/natural_prof.py 8192 1 1 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  python3 - $d $g <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("k_lzsort")]
print("grid %s: k_lzsort FETCH_SIZE %.0f MB per launch (x2 gfx950 correction)" % (sys.argv[2], sum(v) / len(v) * 1024 / 1e6))
PY
done
