#!/bin/bash
# pool kernels on the shared 32-bit pixel decode: GPU tests, smoke, Inception-v3 / EfficientNet-B0 / ResNet-50 benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 400 python bench.py --model inceptionv3 --batch 128 --image-size 299 > gpurun_out/bench_inc.log 2>&1 && tail -1 gpurun_out/bench_inc.log &&
timeout -k 10 400 python bench.py --model efficientnet-b0 --batch 256 > gpurun_out/bench_eff.log 2>&1 && tail -1 gpurun_out/bench_eff.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench_a.log 2>&1 && tail -1 gpurun_out/bench_a.log
