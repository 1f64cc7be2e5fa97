#!/bin/bash
# EfficientNet-B0 b256: bench + one-step kernel breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --model efficientnet-b0 --batch 256 --steps 20 --warmup 8 > gpurun_out/r2s_b0.log 2>&1 || exit $?
tail -1 gpurun_out/r2s_b0.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2s -o hip -- python3 bench.py --model efficientnet-b0 --batch 256 --steps 3 --warmup 3 > gpurun_out/prof_r2s.log 2>&1 &&
python scripts/step_breakdown.py gpurun_out/prof_r2s/hip_kernel_trace.csv > gpurun_out/r2s_step_breakdown.txt && head -40 gpurun_out/r2s_step_breakdown.txt
