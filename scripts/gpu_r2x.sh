#!/bin/bash
# full GPU suite + smoke, then every model family's bench line (one box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || exit $?
bash scripts/gpu_models.sh
