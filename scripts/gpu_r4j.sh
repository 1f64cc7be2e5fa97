#!/bin/bash
# multi-rank rehearsal of the driver's N>1 bench path on one GPU (ranks share the card, gradients over
# gloo, SyncBN over the one-shot peer kernel): 2 ranks at the default b1024, 4 ranks at b256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do sleep 30; date +%s >> gpurun_out/r4j_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 3 --dist-backend gloo > gpurun_out/r4j_2ranks.log 2>&1; rc=$?
echo "2 ranks rc=$rc"; grep -hE "metric|Error|error|peer" gpurun_out/r4j_2ranks.log | cut -c1-400 | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 4 --steps 5 --warmup 3 --batch 256 --dist-backend gloo > gpurun_out/r4j_4ranks.log 2>&1; rc=$?
echo "4 ranks rc=$rc"; grep -hE "metric|Error|error|peer" gpurun_out/r4j_4ranks.log | cut -c1-400 | head -5; exit $rc
