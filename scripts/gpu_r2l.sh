#!/bin/bash
# peer all-reduce tests (2 and 4 ranks on one GPU + ResNet-50 SyncBN step) after the re-entry check
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
bash scripts/gpu_r2k.sh || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_peer.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r2l_peer.log 2>&1; rc=$?; tail -15 gpurun_out/r2l_peer.log; exit $rc
