#!/bin/bash
# Inception numerics (blocks + model) and an on-box A/B of IMGCLS_POOL_CONV_SWAP
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "incep or Incep" --timeout 120 --timeout-method thread > gpurun_out/pytest_inc.log 2>&1 || { tail -40 gpurun_out/pytest_inc.log; exit 1; }
tail -1 gpurun_out/pytest_inc.log
for f in 0 1 0 1; do
  IMGCLS_POOL_CONV_SWAP=$f timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8 > gpurun_out/abp_$f.log 2>&1 || exit $?
  echo "inc swap=$f $(tail -1 gpurun_out/abp_$f.log | cut -c70-110)"
done
