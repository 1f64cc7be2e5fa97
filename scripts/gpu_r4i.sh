#!/bin/bash
# b1536 steady state: tune once (saving the choices), then a kernel trace of 2 steps with those choices
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r4i_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4i_pytest.log 2>&1 || { tail -20 gpurun_out/r4i_pytest.log; exit 1; }; tail -1 gpurun_out/r4i_pytest.log
timeout -k 10 600 python bench.py --batch 1536 --steps 3 --warmup 3 --tune-save gpurun_out/r4i_db1536.json > gpurun_out/r4i_tune.log 2>&1 || { tail -5 gpurun_out/r4i_tune.log; exit 1; }
grep -h metric gpurun_out/r4i_tune.log | cut -c80-200
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b1536s -o hip -- python3 bench.py --batch 1536 --steps 2 --warmup 2 --tune-db gpurun_out/r4i_db1536.json > gpurun_out/r4i_prof.log 2>&1; echo "prof rc=$?"
python scripts/step_breakdown.py gpurun_out/prof_b1536s/hip_kernel_trace.csv > gpurun_out/r4i_b1536_breakdown.txt; head -25 gpurun_out/r4i_b1536_breakdown.txt
python scripts/step_gaps.py gpurun_out/prof_b1536s/hip_kernel_trace.csv | head -12
