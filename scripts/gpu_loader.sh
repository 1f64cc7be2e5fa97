#!/bin/bash
# native loader on the GPU box: GPU numerics test + throughput (uint8 H2D + normalize kernel) vs DataLoader
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -k 10 300 python -u -m pytest tests/test_native_loader.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_loader.log 2>&1; rc=$?
echo "pytest loader rc=$rc"; tail -2 gpurun_out/pytest_loader.log; fatal $rc pytest
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python benchmarks/loader_bench.py --images 4096 --workers 16 --device cuda > gpurun_out/loader_bench.txt 2>&1; rc=$?
echo "loader bench rc=$rc"; tail -1 gpurun_out/loader_bench.txt; fatal $rc loader_bench
