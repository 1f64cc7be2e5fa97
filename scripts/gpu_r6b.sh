#!/bin/bash
# Round 3 call r6b: halo-patch conv kernel (csrc/conv_halo.hip) numerics on every configuration, per-shape
# timing against the LDS-DMA implicit GEMM, and the r5g failures after the same-state test fix.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_hip_ops.py -k "halo" > gpurun_out/r6b_pytest_halo.log 2>&1; rc=$?
tail -4 gpurun_out/r6b_pytest_halo.log
case $rc in 0|1) ;; *) echo "halo tests rc=$rc"; exit 1;; esac
for shape in 64,64,3,1,1,56 128,128,3,1,1,28 256,256,3,1,1,14 512,512,3,1,1,7; do
  for op in fwd dgrad; do
    timeout -k 10 120 python3 scripts/conv_probe.py --batch 1024 --iters 10 --op $op --shape $shape --cfg 1 2>&1 | grep -h " us " || exit 1
    for h in 0 1 2 3 4 5 6 7 8 9 10; do
      timeout -k 10 120 python3 scripts/conv_probe.py --batch 1024 --iters 10 --op $op --shape $shape --halo $h 2>&1 | grep -h " us " || exit 1
    done
  done
done | tee gpurun_out/r6b_halo_probe.txt
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_hip_blocks.py \
  tests/test_gpu_learning.py > gpurun_out/r6b_pytest_blocks.log 2>&1; rc=$?
tail -12 gpurun_out/r6b_pytest_blocks.log
