#!/bin/bash
# Round 3 call r6i: Infinity-Cache reuse probe - a conv's dgrad + wgrad over the whole batch vs per image chunk.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for shape in 64,256,1,1,0,56 256,64,1,1,0,56 128,512,1,1,0,28 64,64,3,1,1,56 256,1024,1,1,0,14; do
  timeout -k 10 180 python3 scripts/mall_probe.py --shape $shape --batch 1024 --chunks 1,2,4,8,16,32 || exit 1
done | tee gpurun_out/r6i_mall_probe.txt
