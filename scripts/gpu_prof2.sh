#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_hip.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_hip.log; fatal $rc bench
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_hip2" -o hip -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > gpurun_out/prof_hip2.log 2>&1; rc=$?
echo "prof rc=$rc"; fatal $rc prof
timeout -k 10 400 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 10 --warmup 3 > gpurun_out/bench_inc.log 2>&1; rc=$?
echo "inception rc=$rc"; tail -3 gpurun_out/bench_inc.log; fatal $rc inc
timeout -k 10 400 python bench.py --model efficientnet-b0 --image-size 224 --batch 256 --steps 10 --warmup 3 > gpurun_out/bench_b0.log 2>&1; rc=$?
echo "effnet rc=$rc"; tail -3 gpurun_out/bench_b0.log; fatal $rc b0
timeout -k 10 400 python bench.py --model efficientnet-b0 --compute torch --image-size 224 --batch 256 --steps 10 --warmup 3 > gpurun_out/bench_b0_torch.log 2>&1; rc=$?
echo "effnet torch rc=$rc"; tail -1 gpurun_out/bench_b0_torch.log; fatal $rc b0t
timeout -k 10 400 python bench.py --model inceptionv3 --compute torch --image-size 299 --batch 128 --steps 10 --warmup 3 > gpurun_out/bench_inc_torch.log 2>&1; rc=$?
echo "inception torch rc=$rc"; tail -1 gpurun_out/bench_inc_torch.log; fatal $rc inct
