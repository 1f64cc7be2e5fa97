#!/bin/bash
# Round 3 call r6d: Inception-v3 b32 graph replay (inf loss in r6c warmup: reproduce or not), eager b32,
# b64 auto, and the headline bench with the stem weight gradient on the compute stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r6d_$tag.log 2>&1 || { tail -3 gpurun_out/r6d_$tag.log; return 0; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r6d_$tag.log | cut -c80-150)"; }
b device --warmup 8 --steps 20
b incep_b32_eager --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 60 --graph off
b incep_b32_a --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 60
b incep_b32_b --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 60
IMGCLS_HALO=0 b incep_b32_nohalo --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 60
b incep_b64 --model inceptionv3 --image-size 299 --batch 64 --warmup 10 --steps 40
b incep_b64_eager --model inceptionv3 --image-size 299 --batch 64 --warmup 10 --steps 40 --graph off
