#!/bin/bash
# full-step kernel trace + breakdown and per-GEMM roofline (all launches)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2i -o hip -- python3 bench.py --steps 3 --warmup 3 --tune-db none > gpurun_out/prof_r2i.log 2>&1 &&
python scripts/step_breakdown.py gpurun_out/prof_r2i/hip_kernel_trace.csv > gpurun_out/r2i_step_breakdown.txt && head -40 gpurun_out/r2i_step_breakdown.txt &&
timeout -k 10 400 python scripts/conv_roofline.py 512 > gpurun_out/r2i_roofline.txt 2>&1 && grep -A4 'roofline at' gpurun_out/r2i_roofline.txt
