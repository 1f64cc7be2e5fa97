#!/bin/bash
# wgrad loader rework: conv tests, conv bench, bench with the committed db vs fresh tuning (alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_ops.py tests/test_hip_blocks.py -x -q --timeout 120 --timeout-method thread -k "conv or stem or wgrad or deterministic or arena or side_stream" > gpurun_out/r2e_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2e_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/conv_bench.py --batch 512 > gpurun_out/r2e_conv_bench.txt 2>&1 && grep -v '^{' gpurun_out/r2e_conv_bench.txt | grep -v amdgpu | head -24 || exit 1
for r in 1 2; do for db in none default; do
  if [ $db = none ]; then X="--tune-db none"; else X=""; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 $X > gpurun_out/r2e_bench.log 2>&1 || exit $?
  echo "db=$db $(tail -1 gpurun_out/r2e_bench.log | grep -o '"value": [0-9.]*')"
done; done
