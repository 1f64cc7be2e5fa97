#!/bin/bash
# specialised branch-free conv epilogues: conv / block tests, per-shape bench, bench, per-GEMM roofline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_ops.py tests/test_hip_blocks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2j_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r2j_pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --tune-db none > gpurun_out/r2j_bench.log 2>&1 || exit $?
  echo "tuned $(tail -1 gpurun_out/r2j_bench.log | grep -o '"value": [0-9.]*')"
done
timeout -k 10 400 python scripts/conv_roofline.py 512 > gpurun_out/r2j_roofline.txt 2>&1 && grep -A4 'roofline at' gpurun_out/r2j_roofline.txt
