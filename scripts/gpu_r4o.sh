#!/bin/bash
# final .so check: GPU suite + smoke
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4o_pytest.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r4o_pytest.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/r4o_pytest.log | tail -1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4o_smoke.log 2>&1 && tail -1 gpurun_out/r4o_smoke.log
