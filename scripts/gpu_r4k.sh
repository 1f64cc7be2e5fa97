#!/bin/bash
# this round's build on every model family (scripts/gpu_models.sh), plus larger per-GPU batches for the
# launch-bound models (Inception-v3 b256, EfficientNet-B0 b512)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
( while true; do sleep 30; date +%s >> gpurun_out/r4k_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
bash scripts/gpu_models.sh || exit $?
for spec in "inception256 --model inceptionv3 --image-size 299 --batch 256" "effb0_512 --model efficientnet-b0 --image-size 224 --batch 512"; do
  set -- $spec; name=$1; shift
  timeout -k 10 500 python bench.py "$@" --steps 20 --warmup 8 > gpurun_out/bench_$name.log 2>&1; rc=$?
  echo "$name rc=$rc"; tail -1 gpurun_out/bench_$name.log | cut -c1-220; [ $rc -eq 0 ] || exit $rc
done
