#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
AMD_SERIALIZE_KERNEL=3 timeout -k 10 600 python -m pytest tests/test_hip_ops.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; fatal $rc pytest
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -m pytest tests/test_gpu_multirank.py -x -q -m gpu > gpurun_out/pytest_multirank.log 2>&1; rc=$?
echo "multirank rc=$rc"; tail -4 gpurun_out/pytest_multirank.log; fatal $rc multirank
timeout -k 10 600 python benchmarks/conv_bench.py --batch 256 --wvariants 1,2 --wblocks 256,512,1024,2048 > gpurun_out/conv_w.log 2>&1; rc=$?
echo "conv_bench rc=$rc"; grep -v '^{' gpurun_out/conv_w.log | tail -48; fatal $rc conv_bench
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_hip.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_hip.log; fatal $rc bench
timeout -k 10 400 python bench.py --model efficientnet-b0 --batch 256 --steps 10 --warmup 3 > gpurun_out/bench_b0.log 2>&1; rc=$?
echo "effnet rc=$rc"; tail -1 gpurun_out/bench_b0.log; fatal $rc b0
