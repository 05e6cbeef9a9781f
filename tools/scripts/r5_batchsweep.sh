#!/bin/bash
# Round 5: batched bench configurations at 4 (HIP default) and 20 hardware queues (GPU box).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/${1:-r5k}_sweep.txt; : > $out
# CFGS: queues:slots:batch tokens
for cfg in ${CFGS:-4:4:5 4:4:4 4:8:3 4:4:8 4:2:10 4:8:2 20:10:2 20:20:1 20:5:4}; do
  set -- ${cfg//:/ }
  extra="--batch $3"
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --hw-queues $1 --inflight $2 $extra --batch-only --no-legs \
    --no-cpu-baseline --no-config2 --no-pmc > gpurun_out/bs.json 2> gpurun_out/bs.err
  rc=$?
  if [ $rc != 0 ]; then echo "q$1 d$2 b$3 FAILED rc=$rc: $(tail -c 600 gpurun_out/bs.err | tr '\n' ' ')" >> $out; [ $rc = 3 ] || { cat $out; exit 1; }; continue; fi
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/bs.json').read().strip().splitlines()[-1])
print('queues $1 slots $2 batch $3: %.1f GB/s  %s' % (d['value']/1e3, d['detail'].get('slot_files_bit_exact')))" >> $out
done
cat $out
