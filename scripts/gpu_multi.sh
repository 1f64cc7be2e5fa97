#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 at $2"; exit "$1";; esac; }
timeout -k 10 300 python bench.py --steps 10 --warmup 5 > gpurun_out/bench1.log 2>&1; rc=$?
echo "bench1 rc=$rc"; grep -E "host enqueue|metric" gpurun_out/bench1.log | cut -c1-200; fatal $rc bench1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 3 --batch 64 --dist-backend gloo > gpurun_out/bench2_gloo.log 2>&1; rc=$?
echo "bench2(gloo, shared GPU) rc=$rc"; grep -E "host enqueue|metric|Error|error" gpurun_out/bench2_gloo.log | cut -c1-250 | head; fatal $rc bench2
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 train.py --synthetic --model resnet18 --image-size 64 --batchsize 32 --epochs 2 --synthetic-train-size 256 --synthetic-val-size 64 --num-workers 2 --backend gloo --ckpt-dir /tmp/ck_gpu --no-progress --val-batchsize 16 --resume none > gpurun_out/train2_gloo.log 2>&1; rc=$?
echo "train2 rc=$rc"; grep -E "Validation|improved|Error" gpurun_out/train2_gloo.log | head; fatal $rc train2
