#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -x -q -k "fp8 or mx" --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1; rc=$?
echo "pytest fp8 rc=$rc"; tail -2 gpurun_out/pytest_fp8.log; fatal $rc pytest
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --dtype fp8 --steps 20 --warmup 8 > gpurun_out/bench_fp8.log 2>&1; rc=$?
echo "bench fp8 rc=$rc"; tail -1 gpurun_out/bench_fp8.log | cut -c1-250; fatal $rc bench
