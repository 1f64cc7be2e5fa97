#!/bin/bash
# 512-B-row transposed-read swizzle: wgrad tests + wgrad tuning log on the big shapes + bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_ops.py -x -q --timeout 120 --timeout-method thread -k "wgrad_ring or conv_fwd_bwd" > gpurun_out/r2g_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r2g_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python benchmarks/conv_bench.py --batch 512 --tune-log > gpurun_out/r2g_conv_bench.txt 2>&1 && grep "wgrad Co\|x[0-9]:" gpurun_out/r2g_conv_bench.txt | cut -c1-400 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --tune-db none > gpurun_out/r2g_bench.log 2>&1 || exit $?
  echo "tuned $(tail -1 gpurun_out/r2g_bench.log | grep -o '"value": [0-9.]*')"
done
