#!/bin/bash
# Same-box HIP vs reference-stack (torch DDP + MIOpen, bf16 autocast) ResNet-50 b1024 bench; a ticker keeps the
# job visibly alive while MIOpen's find step runs silently.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/refstack_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 300 python bench.py --warmup 8 --steps 20 > gpurun_out/r13b_hip.log 2>&1 || exit 1
grep -h '^{"metric' gpurun_out/r13b_hip.log | grep -o '"value": [0-9.]*'
timeout -k 10 900 python bench.py --compute torch --warmup 8 --steps 20 > gpurun_out/r13b_torch.log 2>&1 || { tail -3 gpurun_out/r13b_torch.log; exit 1; }
grep -h '^{"metric' gpurun_out/r13b_torch.log | grep -o '"value": [0-9.]*'
timeout -k 10 600 python bench.py --compute torch --model inceptionv3 --image-size 299 --batch 128 --warmup 8 --steps 20 > gpurun_out/r13b_torch_incep.log 2>&1 || { tail -3 gpurun_out/r13b_torch_incep.log; exit 1; }
grep -h '^{"metric' gpurun_out/r13b_torch_incep.log | grep -o '"value": [0-9.]*'
