#!/bin/bash
# fused SyncBN peer kernels: peer tests (2/4 ranks, ResNet-50 SyncBN step vs torch.distributed), multi-rank
# GPU tests, 2-rank bench rehearsal (peer vs gloo)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_multirank.py -x -v --timeout 180 --timeout-method thread > gpurun_out/r2y_pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" gpurun_out/r2y_pytest.log | tail -12
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r2y_pytest.log | head -20; exit $rc; }
bash scripts/gpu_r2m.sh
