#!/bin/bash
# conv kernel tests + per-shape microbenchmark with optional A/B flags (CONV_ARGS)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -k 10 400 python -m pytest tests/test_hip_ops.py -x -q -m gpu -k "conv" > gpurun_out/pytest_conv.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_conv.log; fatal $rc pytest
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python benchmarks/conv_bench.py $CONV_ARGS > gpurun_out/conv_bench.txt 2>&1; rc=$?
echo "conv_bench rc=$rc"; tail -4 gpurun_out/conv_bench.txt; fatal $rc conv_bench
