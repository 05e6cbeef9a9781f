set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/g12; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['detail'].get('natural_s0_single_MBps'), d['detail'].get('natural_s0_MBps'))"
