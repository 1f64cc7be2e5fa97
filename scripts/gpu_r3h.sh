#!/bin/bash
# full GPU suite (incl. the HIP-graph equality tests) + smoke + ResNet-50 headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3h_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r3h_pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3h_pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3h_smoke.log 2>&1 && tail -1 gpurun_out/r3h_smoke.log || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r3h_bench.log 2>&1 && tail -1 gpurun_out/r3h_bench.log
MODEL=inceptionv3 RES=299 BATCH=128 bash scripts/gpu_prof_model.sh && python scripts/step_breakdown.py gpurun_out/prof_inceptionv3/hip_kernel_trace.csv > gpurun_out/r3h_inception_step_breakdown.txt && head -30 gpurun_out/r3h_inception_step_breakdown.txt
