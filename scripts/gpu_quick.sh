#!/bin/bash
# tests + 1-GPU bench (+ optional extra bench args via BENCH_ARGS)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; fatal $rc pytest
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --batch 256 $BENCH_ARGS > gpurun_out/bench_hip.log 2>&1; rc=$?
echo "bench rc=$rc"; grep -h "host enqueue" gpurun_out/bench_hip.log; tail -1 gpurun_out/bench_hip.log; fatal $rc bench
timeout -k 10 300 python bench.py > gpurun_out/bench_hip512.log 2>&1; rc=$?
echo "bench512 rc=$rc"; tail -1 gpurun_out/bench_hip512.log; fatal $rc bench512
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_q" -o hip -- python3 "$ROOT/bench.py" --batch 256 --steps 5 --warmup 3 > gpurun_out/prof_q.log 2>&1; rc=$?
echo "prof rc=$rc"; fatal $rc prof
