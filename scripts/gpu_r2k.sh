#!/bin/bash
# Re-entry check of HEAD: full GPU tests, smoke, default bench (committed find-db) vs freshly tuned
# choices (saved for a db refresh), one-step kernel trace + breakdown.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/db
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 && echo "db   $(tail -1 gpurun_out/bench_default.log)" || exit $?
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --tune-db none --tune-save gpurun_out/db/r50_$r.json > gpurun_out/db/r50_$r.log 2>&1 || exit $?
  echo "tuned $r $(tail -1 gpurun_out/db/r50_$r.log | grep -o '"value": [0-9.]*')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2k -o hip -- python3 bench.py --steps 3 --warmup 3 --tune-db gpurun_out/db/r50_1.json > gpurun_out/prof_r2k.log 2>&1 &&
python scripts/step_breakdown.py gpurun_out/prof_r2k/hip_kernel_trace.csv > gpurun_out/r2k_step_breakdown.txt && head -40 gpurun_out/r2k_step_breakdown.txt
