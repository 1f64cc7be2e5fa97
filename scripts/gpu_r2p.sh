#!/bin/bash
# fp8 vs bf16 on this build: retuned benches + one-step kernel trace of the fp8 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/db
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench.py --dtype fp8 --steps 20 --warmup 8 --tune-db none --tune-save gpurun_out/db/r2p_fp8_$r.json > gpurun_out/r2p_fp8_$r.log 2>&1 || exit $?
  echo "fp8 $r $(tail -1 gpurun_out/r2p_fp8_$r.log | grep -o '"value": [0-9.]*')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2p -o hip -- python3 bench.py --dtype fp8 --steps 3 --warmup 3 --tune-db gpurun_out/db/r2p_fp8_1.json > gpurun_out/prof_r2p.log 2>&1 &&
python scripts/step_breakdown.py gpurun_out/prof_r2p/hip_kernel_trace.csv > gpurun_out/r2p_step_breakdown.txt && head -30 gpurun_out/r2p_step_breakdown.txt
