#!/bin/bash
# 32-row wgrad tile: numerics, then Inception / EfficientNet-B0 throughput (the tuner picks per shape)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -x -q -m gpu -k "conv or wgrad" --timeout 120 --timeout-method thread > gpurun_out/pytest_wg32.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_wg32.log; [ $rc -eq 0 ] || { grep -E "^E|FAILED" gpurun_out/pytest_wg32.log | head; exit 1; }
for i in 1 2; do timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 30 --warmup 10 > gpurun_out/bench_inc.log 2>&1 && tail -1 gpurun_out/bench_inc.log | cut -c60-110; done
timeout -k 10 300 python bench.py --model efficientnet-b0 --image-size 224 --batch 256 --steps 20 --warmup 8 > gpurun_out/bench_effb0.log 2>&1 && tail -1 gpurun_out/bench_effb0.log | cut -c60-110
