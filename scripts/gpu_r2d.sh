#!/bin/bash
# conv kernel rework: conv numerics tests, plain-GEMM reference, per-shape conv bench, default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_ops.py -x -q --timeout 120 --timeout-method thread -k "conv or stem or fp8 or dense" > gpurun_out/r2d_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2d_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/gemm_ref.py > gpurun_out/r2d_gemm_ref.txt 2>&1 && grep -v amdgpu gpurun_out/r2d_gemm_ref.txt &&
timeout -k 10 300 python benchmarks/conv_bench.py --batch 512 > gpurun_out/r2d_conv_bench.txt 2>&1 && grep -v '^{' gpurun_out/r2d_conv_bench.txt | grep -v amdgpu | head -30 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2d_bench.log 2>&1 && tail -1 gpurun_out/r2d_bench.log | cut -c1-150
