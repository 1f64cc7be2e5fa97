#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -x -q -k "bn" --timeout 120 --timeout-method thread > gpurun_out/pytest_bn.log 2>&1; rc=$?
echo "pytest bn rc=$rc"; tail -2 gpurun_out/pytest_bn.log; fatal $rc pytest
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python benchmarks/bn_bench.py --batch 512 > gpurun_out/bn_bench.txt 2>&1; rc=$?
echo "bn bench rc=$rc"; cat gpurun_out/bn_bench.txt | cut -c1-250; fatal $rc bn_bench
