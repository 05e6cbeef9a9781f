#!/bin/bash
# Runs the encoder parity tests against each prebuilt library variant in variants/ (measurement).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cp hoh-ans_amd/lib/libhohgpu.so /tmp/orig.so
for v in variants/*.so; do
  cp $v hoh-ans_amd/lib/libhohgpu.so
  echo "== $v"; timeout -k 10 200 python -u -m pytest tests/test_gpu_encode.py -q -m gpu --timeout 120 --timeout-method thread -s -k "${VK:-}" > gpurun_out/var.log 2>&1; grep -E "FAILED|passed|failed" gpurun_out/var.log; grep -E "^[FB] t=" gpurun_out/var.log | head -${VN:-20}
done
cp /tmp/orig.so hoh-ans_amd/lib/libhohgpu.so
