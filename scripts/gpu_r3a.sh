#!/bin/bash
# U-row BN elementwise kernels: BN / block tests, then ResNet-50 b512 and EfficientNet-B0 A/B (alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_ops.py tests/test_hip_blocks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r3a_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r3a_pytest.log | head -20; exit $rc; }
for r in 1 2; do
  for u in 0 1; do
    IMGCLS_BN_UNROLL=$u timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/r3a_r50_$u.log 2>&1 || exit $?
    echo "r50 unroll=$u $(tail -1 gpurun_out/r3a_r50_$u.log | grep -o '"value": [0-9.]*')"
  done
done
for u in 0 1; do
  IMGCLS_BN_UNROLL=$u timeout -k 10 300 python bench.py --model efficientnet-b0 --batch 256 --steps 20 --warmup 8 > gpurun_out/r3a_b0_$u.log 2>&1 || exit $?
  echo "b0 unroll=$u $(tail -1 gpurun_out/r3a_b0_$u.log | grep -o '"value": [0-9.]*')"
done
