#!/bin/bash
# GPU tests + rocprofv3 kernel statistics of the HIP and reference-stack training steps.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; fatal $rc pytest
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_hip" -o hip -- python3 "$ROOT/bench.py" --compute hip --steps 5 --warmup 2 > gpurun_out/prof_hip.log 2>&1; rc=$?
echo "prof hip rc=$rc"; tail -2 gpurun_out/prof_hip.log; fatal $rc prof_hip
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_torch" -o torch -- python3 "$ROOT/bench.py" --compute torch --steps 5 --warmup 2 > gpurun_out/prof_torch.log 2>&1; rc=$?
echo "prof torch rc=$rc"; tail -2 gpurun_out/prof_torch.log; fatal $rc prof_torch
for b in 128 384; do
timeout -k 10 300 python bench.py --compute hip --steps 10 --warmup 3 --batch $b > gpurun_out/bench_hip_b$b.log 2>&1; rc=$?
echo "bench hip b$b rc=$rc"; tail -1 gpurun_out/bench_hip_b$b.log; fatal $rc bench
done
exit 0
