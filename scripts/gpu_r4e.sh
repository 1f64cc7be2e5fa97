#!/bin/bash
# Inception-v3 b128 (the reference's default model): kernel trace, per-queue idle gaps, host-side profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
MODEL=inceptionv3 RES=299 BATCH=128 bash scripts/gpu_prof_model.sh && python scripts/step_breakdown.py gpurun_out/prof_inceptionv3/hip_kernel_trace.csv > gpurun_out/r4e_inception_step_breakdown.txt && python scripts/step_gaps.py gpurun_out/prof_inceptionv3/hip_kernel_trace.csv > gpurun_out/r4e_inception_gaps.txt && cat gpurun_out/r4e_inception_gaps.txt && head -5 gpurun_out/r4e_inception_step_breakdown.txt
