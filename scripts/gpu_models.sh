#!/bin/bash
# 1-GPU throughput of the other model families (same bench harness, synthetic data)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > "gpurun_out/bench_$name.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 "gpurun_out/bench_$name.log" | cut -c1-220; fatal $rc "$name"
}
run inception --model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8
run effb0 --model efficientnet-b0 --image-size 224 --batch 256 --steps 20 --warmup 8
run r101 --model resnet101 --image-size 224 --batch 256 --steps 15 --warmup 6
run effb3 --model efficientnet-b3 --image-size 300 --batch 128 --steps 15 --warmup 6
run r50fp8 --dtype fp8 --steps 20 --warmup 8
run r50 --steps 20 --warmup 8
run r50b256 --batch 256 --steps 20 --warmup 8
