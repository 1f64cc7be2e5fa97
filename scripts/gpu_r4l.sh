#!/bin/bash
# larger batches for the launch-bound models and the reference stack at the batches the README quotes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
( while true; do sleep 30; date +%s >> gpurun_out/r4l_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
for spec in "inception512 --model inceptionv3 --image-size 299 --batch 512" "effb0_1024 --model efficientnet-b0 --image-size 224 --batch 1024" \
            "torch_inception256 --model inceptionv3 --image-size 299 --batch 256 --compute torch" \
            "torch_effb0_512 --model efficientnet-b0 --image-size 224 --batch 512 --compute torch"; do
  set -- $spec; name=$1; shift
  timeout -k 10 600 python bench.py "$@" --steps 15 --warmup 6 > gpurun_out/bench_$name.log 2>&1; rc=$?
  echo "$name rc=$rc"; tail -1 gpurun_out/bench_$name.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
