#!/bin/bash
# channel-fixed BN elementwise kernels: GPU tests, BN bandwidth table, headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 300 python benchmarks/bn_bench.py --batch 512 > gpurun_out/bn_bench.txt 2>&1 && cut -c1-250 gpurun_out/bn_bench.txt &&
timeout -k 10 400 python bench.py > gpurun_out/bench_a.log 2>&1 && tail -1 gpurun_out/bench_a.log &&
timeout -k 10 400 python bench.py --model inceptionv3 --batch 128 --image-size 299 > gpurun_out/bench_inc.log 2>&1 && tail -1 gpurun_out/bench_inc.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench_b.log 2>&1 && tail -1 gpurun_out/bench_b.log
