#!/bin/bash
# Reusable: bench.py over the model zoo on one GPU box (README results table).  TAG names the outputs.
#   gpurun --timeout 1200 -- 'TAG=r7b bash scripts/bench_models.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-models}
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/${T}_$tag.log 2>&1 || { tail -3 gpurun_out/${T}_$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/${T}_$tag.log | grep -o '"value": [0-9.]*')"; }
b resnet50_b1024 --batch 1024 --warmup 5 --steps 20 || exit 1
b resnet50_b1024_host --batch 1024 --warmup 5 --steps 20 --data host || exit 1
b resnet50_b256 --batch 256 --warmup 8 --steps 20 || exit 1
b resnet50_b512 --batch 512 --warmup 8 --steps 20 || exit 1
b resnet101_b256 --model resnet101 --batch 256 --warmup 8 --steps 20 || exit 1
b incep_b4 --model inceptionv3 --image-size 299 --batch 4 --warmup 10 --steps 60 || exit 1
b incep_b32 --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 40 || exit 1
b incep_b128 --model inceptionv3 --image-size 299 --batch 128 --warmup 8 --steps 20 || exit 1
b incep_b256 --model inceptionv3 --image-size 299 --batch 256 --warmup 8 --steps 20 || exit 1
b incep_b512 --model inceptionv3 --image-size 299 --batch 512 --warmup 8 --steps 20 || exit 1
b effb0_b256 --model efficientnet-b0 --batch 256 --warmup 8 --steps 20 || exit 1
b effb0_b512 --model efficientnet-b0 --batch 512 --warmup 8 --steps 20 || exit 1
b effb0_b1024 --model efficientnet-b0 --batch 1024 --warmup 8 --steps 20 || exit 1
b effb3_b128 --model efficientnet-b3 --image-size 300 --batch 128 --warmup 8 --steps 20 || exit 1
