#!/bin/bash
# Round-2 first GPU pass: GPU tests, smoke, default bench, one-step kernel trace + breakdown,
# per-GEMM roofline of the ResNet-50 b512 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -2 gpurun_out/pytest_gpu.log &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2a -o hip -- python3 bench.py --steps 3 --warmup 3 > gpurun_out/prof_r2a.log 2>&1 &&
python scripts/step_breakdown.py gpurun_out/prof_r2a/hip_kernel_trace.csv > gpurun_out/r2a_step_breakdown.txt && head -30 gpurun_out/r2a_step_breakdown.txt &&
timeout -k 10 400 python scripts/conv_roofline.py 512 > gpurun_out/r2a_roofline.txt 2>&1 && grep -A4 'roofline at' gpurun_out/r2a_roofline.txt
