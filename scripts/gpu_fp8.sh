#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
for B in 256 512; do
  timeout -k 10 300 python bench.py --batch $B --dtype fp8 > gpurun_out/bench_fp8_$B.log 2>&1; rc=$?
  echo "fp8 b$B rc=$rc"; tail -1 gpurun_out/bench_fp8_$B.log | cut -c1-200; fatal $rc fp8
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_fp8" -o hip -- python3 "$ROOT/bench.py" --batch 256 --dtype fp8 --steps 4 --warmup 3 > gpurun_out/prof_fp8.log 2>&1; rc=$?
echo "prof rc=$rc"; fatal $rc prof
