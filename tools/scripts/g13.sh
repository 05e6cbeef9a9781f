set -o pipefail
# in-flight sweep of the driver-shaped command (20 steps, 5 warmup), two runs each
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/g13; mkdir -p $O; export TMPDIR=/tmp
for d in 12 16 20 24; do
  for r in 1 2; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --inflight $d --no-cpu-baseline --no-pmc --no-config2 --no-legs > $O/b_${d}_$r.json 2> $O/b_${d}_$r.err || { tail -5 $O/b_${d}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b_${d}_$r.json').read().strip().splitlines()[-1]); print($d, $r, d['value'])"
  done
done
