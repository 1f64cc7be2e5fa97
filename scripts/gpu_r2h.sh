#!/bin/bash
# wgrad split-K workspace: tests, per-shape tuning (ws vs atomics), bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_ops.py tests/test_hip_blocks.py -x -q --timeout 120 --timeout-method thread -k "wgrad or conv_fwd_bwd or side_stream or deterministic" > gpurun_out/r2h_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r2h_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python benchmarks/conv_bench.py --batch 512 --tune-log > gpurun_out/r2h_conv_bench.txt 2>&1 && grep "x[0-9]:" gpurun_out/r2h_conv_bench.txt | cut -c1-140 && grep "tuned wgrad" gpurun_out/r2h_conv_bench.txt || exit 1
for r in 1 2; do for v in 0 1; do
  IMGCLS_WGRAD_WS=$v timeout -k 10 300 python bench.py --steps 20 --warmup 8 --tune-db none > gpurun_out/r2h_bench.log 2>&1 || exit $?
  echo "ws=$v $(tail -1 gpurun_out/r2h_bench.log | grep -o '"value": [0-9.]*')"
done; done
