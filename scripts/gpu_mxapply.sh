#!/bin/bash
# channel-fixed MX-FP8 BN apply: GPU tests, fp8 and bf16 ResNet-50 benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 400 python bench.py --dtype fp8 > gpurun_out/bench_fp8.log 2>&1 && tail -1 gpurun_out/bench_fp8.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench_a.log 2>&1 && tail -1 gpurun_out/bench_a.log
