#!/bin/bash
# fused stem BN-ReLU-maxpool with 32-bit index math: GPU tests, rocprofv3 kernel stats of the
# ResNet-50 b512 step, headline bench A/B pair, EfficientNet-B0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; ROOT="$(pwd)"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_r1f" -o hip -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > gpurun_out/prof_r1f.log 2>&1 && tail -1 gpurun_out/prof_r1f.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench_a.log 2>&1 && tail -1 gpurun_out/bench_a.log &&
timeout -k 10 400 python bench.py --model efficientnet-b0 --batch 256 > gpurun_out/bench_eff.log 2>&1 && tail -1 gpurun_out/bench_eff.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench_b.log 2>&1 && tail -1 gpurun_out/bench_b.log
