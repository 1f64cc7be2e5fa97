#!/bin/bash
# A/B of the fused stem (BN-act-maxpool) on one box + a kernel trace of the fused step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -k "pool" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pool.log 2>&1 || { tail -30 gpurun_out/pytest_pool.log; exit 1; }
for f in 0 1 0 1; do
  IMGCLS_STEM_POOL_FUSE=$f timeout -k 10 300 python bench.py --batch 256 --steps 20 --warmup 8 > gpurun_out/ab_$f.log 2>&1 || exit $?
  echo "r50 fuse=$f $(tail -1 gpurun_out/ab_$f.log | cut -c80-120)"
done
for f in 0 1; do
  IMGCLS_STEM_POOL_FUSE=$f timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8 > gpurun_out/abi_$f.log 2>&1 || exit $?
  echo "inc fuse=$f $(tail -1 gpurun_out/abi_$f.log | cut -c70-120)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pool -o run --output-format csv -- python bench.py --batch 256 --steps 4 --warmup 4 > gpurun_out/prof_pool.log 2>&1
