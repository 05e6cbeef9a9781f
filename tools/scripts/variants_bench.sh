#!/bin/bash
# Bench each prebuilt library variant in variants/ (alternating, two rounds); parity tests on the
# first.  Measurement only: the tree's own library is restored afterwards.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cp hoh-ans_amd/lib/libhohgpu.so /tmp/orig.so
first=$(ls variants/*.so | head -1)
cp $first hoh-ans_amd/lib/libhohgpu.so
timeout -k 10 400 python -u -m pytest ${VT:-tests/test_gpu_encode.py} -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -20 gpurun_out/t.log; cp /tmp/orig.so hoh-ans_amd/lib/libhohgpu.so; exit 1; }
echo "$first: $(tail -1 gpurun_out/t.log)"
for r in 1 2; do
  for v in variants/*.so; do
    cp $v hoh-ans_amd/lib/libhohgpu.so
    timeout -k 5 300 python bench.py --no-cpu-baseline > gpurun_out/vb.json 2>gpurun_out/vb.err || { tail -5 gpurun_out/vb.err; break; }
    python -c "import json;d=json.load(open('gpurun_out/vb.json'));print('$v', d['value'], d['detail']['kernel_avg_ms_one_in_flight'].get('front') if 'kernel_avg_ms_one_in_flight' in d['detail'] else '')"
  done
done
cp /tmp/orig.so hoh-ans_amd/lib/libhohgpu.so
