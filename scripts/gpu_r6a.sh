#!/bin/bash
# Round 3 call r6a: the GPU tests that failed in r5g after the same-state fix (BN buffers restored between
# compared runs), plus the chain test without the BN statistics pivot for comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
T="tests/test_hip_blocks.py tests/test_gpu_learning.py"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $T > gpurun_out/r6a_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r6a_pytest.log
case $rc in 0|1) ;; *) echo "rc=$rc"; exit 1;; esac
IMGCLS_BN_SHIFT=0 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread \
  "tests/test_hip_blocks.py::test_block_slots" > gpurun_out/r6a_pytest_noshift.log 2>&1
tail -5 gpurun_out/r6a_pytest_noshift.log
