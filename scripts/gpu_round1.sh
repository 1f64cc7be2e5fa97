#!/bin/bash
# GPU pass: kernel numerics, smoke, reference-stack vs HIP bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/dev.txt 2>&1
timeout -k 10 600 python -m pytest tests/test_hip_ops.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 400 python bench.py --compute torch --steps 20 --warmup 5 > gpurun_out/bench_torch.log 2>&1; rc=$?
echo "bench torch rc=$rc"; tail -3 gpurun_out/bench_torch.log; fatal $rc bench_torch
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; fatal $rc smoke
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --compute hip --steps 10 --warmup 3 > gpurun_out/bench_hip.log 2>&1; rc=$?
echo "bench hip rc=$rc"; tail -3 gpurun_out/bench_hip.log; fatal $rc bench_hip
exit 0
