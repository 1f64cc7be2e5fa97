#!/bin/bash
# direct 3x3 conv: numerics, per-shape tuning log (ResNet layer1), Inception + ResNet throughput
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -x -q -m gpu -k "direct or conv_fwd_bwd or stem or conv_bn_act" --timeout 120 --timeout-method thread > gpurun_out/pytest_direct.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_direct.log; [ $rc -eq 0 ] || { grep -E "^E|FAILED" gpurun_out/pytest_direct.log | head; exit 1; }
timeout -k 10 300 python benchmarks/conv_bench.py --batch 512 --tune-log --only 1,2 > gpurun_out/direct_tune.txt 2>&1 || exit $?
grep -E "tune|k3s1" gpurun_out/direct_tune.txt | cut -c1-330
timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8 > gpurun_out/bench_inc.log 2>&1 && tail -1 gpurun_out/bench_inc.log | cut -c60-110
IMGCLS_DIRECT_CONV=0 timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8 > gpurun_out/bench_inc0.log 2>&1 && tail -1 gpurun_out/bench_inc0.log | cut -c60-110
timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_r50.log 2>&1 && tail -1 gpurun_out/bench_r50.log | cut -c80-120
IMGCLS_DIRECT_CONV=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_r50_0.log 2>&1 && tail -1 gpurun_out/bench_r50_0.log | cut -c80-120
