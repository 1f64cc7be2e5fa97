#!/bin/bash
# whole-step HIP graph: bitwise check against eager (deterministic mode, single-stream and side-stream
# capture), a non-deterministic tracking check, then eager vs graph bench A/B on three model families
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
IMGCLS_GRAPH_SIDE=0 timeout -k 10 300 python -u scripts/graph_check.py --model resnet50 --batch 32 --steps 10 --det > gpurun_out/r3f_det_noside.txt 2>&1; echo "det single-stream rc=$? $(tail -1 gpurun_out/r3f_det_noside.txt)"
timeout -k 10 300 python -u scripts/graph_check.py --model resnet50 --batch 32 --steps 10 --det > gpurun_out/r3f_det_side.txt 2>&1; echo "det side-stream rc=$? $(tail -1 gpurun_out/r3f_det_side.txt)"
timeout -k 10 300 python -u scripts/graph_check.py --model resnet50 --batch 64 --steps 12 > gpurun_out/r3f_nondet.txt 2>&1 || exit $?
tail -14 gpurun_out/r3f_nondet.txt
for m in "resnet50 512 224" "inceptionv3 128 299" "efficientnet-b0 256 224"; do
  set -- $m
  for gph in off on; do
    timeout -k 10 300 python bench.py --model $1 --batch $2 --image-size $3 --steps 20 --warmup 8 --graph $gph > gpurun_out/r3f_$1_$gph.log 2>&1 || { tail -5 gpurun_out/r3f_$1_$gph.log; exit 1; }
    echo "$1 graph=$gph $(tail -1 gpurun_out/r3f_$1_$gph.log | grep -o '"value": [0-9.]*') $(grep -o 'host enqueue [0-9.]* ms' gpurun_out/r3f_$1_$gph.log) $(tail -1 gpurun_out/r3f_$1_$gph.log | grep -o '"final_loss": [0-9.e+-]*')"
  done
done
