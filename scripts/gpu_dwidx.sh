#!/bin/bash
# depthwise / SE kernels with 32-bit index math: GPU tests, EfficientNet-B0 / B3 benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 400 python bench.py --model efficientnet-b0 --batch 256 > gpurun_out/bench_eff.log 2>&1 && tail -1 gpurun_out/bench_eff.log &&
timeout -k 10 400 python bench.py --model efficientnet-b3 --image-size 300 --batch 128 --steps 15 --warmup 6 > gpurun_out/bench_eff3.log 2>&1 && tail -1 gpurun_out/bench_eff3.log &&
timeout -k 10 400 python bench.py --model efficientnet-b0 --batch 256 > gpurun_out/bench_eff_b.log 2>&1 && tail -1 gpurun_out/bench_eff_b.log
