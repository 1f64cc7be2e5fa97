#!/bin/bash
# parallel split-K reduce + unrolled BN-backward reduce + 64/128 x 256 wgrad tiles: full GPU suite, bench
# with the committed find-db (old wgrad choices), then with the narrow-Cout wgrad shapes re-timed
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4c_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/r4c_pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r4c_pytest_gpu.log | head; exit $rc; }
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/r4c_bench_db$i.log 2>&1 && tail -1 gpurun_out/r4c_bench_db$i.log | cut -c1-200 || exit $?; done
timeout -k 10 400 python bench.py --tune-db tuning/exp_wide_wgrad_db.json --tune-save gpurun_out/r4c_db.json > gpurun_out/r4c_bench_tune.log 2>&1 && tail -1 gpurun_out/r4c_bench_tune.log | cut -c1-200 || exit $?
for i in 1 2; do timeout -k 10 300 python bench.py --tune-db gpurun_out/r4c_db.json > gpurun_out/r4c_bench_new$i.log 2>&1 && tail -1 gpurun_out/r4c_bench_new$i.log | cut -c1-200 || exit $?; done
timeout -k 10 300 python bench.py > gpurun_out/r4c_bench_db3.log 2>&1 && tail -1 gpurun_out/r4c_bench_db3.log | cut -c1-200 || exit $?
IMGCLS_TUNE_DB=gpurun_out/r4c_db.json MODEL=resnet50 RES=224 BATCH=512 bash scripts/gpu_prof_model.sh && python scripts/step_breakdown.py gpurun_out/prof_resnet50/hip_kernel_trace.csv > gpurun_out/r4c_resnet50_step_breakdown.txt && head -14 gpurun_out/r4c_resnet50_step_breakdown.txt
