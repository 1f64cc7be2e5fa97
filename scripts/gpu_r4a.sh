#!/bin/bash
# re-entry check on a fresh container build: full GPU suite, smoke, headline bench, rocprof step breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r4a_pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r4a_pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.log 2>&1 && tail -1 gpurun_out/r4a_smoke.log || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r4a_bench.log 2>&1 && tail -1 gpurun_out/r4a_bench.log | cut -c1-300 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r4a_bench2.log 2>&1 && tail -1 gpurun_out/r4a_bench2.log | cut -c1-300 || exit $?
MODEL=resnet50 RES=224 BATCH=512 bash scripts/gpu_prof_model.sh && python scripts/step_breakdown.py gpurun_out/prof_resnet50/hip_kernel_trace.csv > gpurun_out/r4a_resnet50_step_breakdown.txt && head -12 gpurun_out/r4a_resnet50_step_breakdown.txt
