#!/bin/bash
# Inception-v3 b128: one-step kernel breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2z -o hip -- python3 bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 3 --warmup 3 > gpurun_out/prof_r2z.log 2>&1 &&
python scripts/step_breakdown.py gpurun_out/prof_r2z/hip_kernel_trace.csv > gpurun_out/r2z_step_breakdown.txt && head -40 gpurun_out/r2z_step_breakdown.txt
