#!/bin/bash
# rocprofv3 kernel trace of the headline config (ResNet-50 b1024, find-db seeded): step breakdown, per-queue gaps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
MODEL=resnet50 RES=224 BATCH=1024 bash scripts/gpu_prof_model.sh || exit 1
python scripts/step_breakdown.py gpurun_out/prof_resnet50/hip_kernel_trace.csv > gpurun_out/r4n_resnet50_b1024_step_breakdown.txt
python scripts/step_gaps.py gpurun_out/prof_resnet50/hip_kernel_trace.csv > gpurun_out/r4n_resnet50_b1024_gaps.txt
head -16 gpurun_out/r4n_resnet50_b1024_step_breakdown.txt; head -4 gpurun_out/r4n_resnet50_b1024_gaps.txt
