#!/bin/bash
# conv tile-config numerics + per-shape benchmark with the tuner's candidate times
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_hip_ops.py -x -q -m gpu -k "conv" --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_conv.log; fatal $rc pytest
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python benchmarks/conv_bench.py --batch ${CONV_BATCH:-512} --tune-log $CONV_ARGS > gpurun_out/conv_tiles.txt 2>&1; rc=$?
echo "conv_bench rc=$rc"; grep -v '^{' gpurun_out/conv_tiles.txt | tail -80; fatal $rc conv_bench
[ "${CONV_BENCH_TOO:-0}" = 1 ] || exit 0
timeout -k 10 400 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_r50.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_r50.log | cut -c1-200; fatal $rc bench
