#!/bin/bash
# N>1 bench rehearsal on one GPU: 2 ranks (gloo for the process group), SyncBN statistics over the
# peer kernel vs over torch.distributed; small batch (functional, not a performance number)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for comm in peer rccl; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 2 --dist-backend gloo --steps 4 --warmup 3 --batch 32 --syncbn-comm $comm > gpurun_out/r2m_$comm.log 2>&1 || { tail -30 gpurun_out/r2m_$comm.log; exit 1; }
  echo "$comm: $(grep metric gpurun_out/r2m_$comm.log)"
done
