#!/bin/bash
# row-strip depthwise kernels: kernel tests, EfficientNet-B0 A/B (row-strip vs per-pixel) + breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dwconv.py tests/test_hip_ops.py -k "depthwise or dw" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2t_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2t_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model efficientnet-b0 --batch 256 --steps 20 --warmup 8 > gpurun_out/r2t_b0.log 2>&1 || exit $?
tail -1 gpurun_out/r2t_b0.log | grep -o '"value": [0-9.]*'
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2t -o hip -- python3 bench.py --model efficientnet-b0 --batch 256 --steps 3 --warmup 3 > gpurun_out/prof_r2t.log 2>&1 &&
python scripts/step_breakdown.py gpurun_out/prof_r2t/hip_kernel_trace.csv > gpurun_out/r2t_step_breakdown.txt && head -24 gpurun_out/r2t_step_breakdown.txt
