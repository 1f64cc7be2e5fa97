#!/bin/bash
# Round 3 call r6f: native RCCL communicator tests (world of one), serialised-vs-concurrent race check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_rccl.py \
  > gpurun_out/r6f_pytest_rccl.log 2>&1; rc=$?
tail -8 gpurun_out/r6f_pytest_rccl.log
case $rc in 0|1) ;; *) echo "rccl tests rc=$rc"; exit 1;; esac
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread tests/test_gpu_race.py \
  > gpurun_out/r6f_pytest_race.log 2>&1; rc=$?
tail -6 gpurun_out/r6f_pytest_race.log
