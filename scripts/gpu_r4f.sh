#!/bin/bash
# per-GPU batch sweep for the headline (ResNet-50 224, one GPU): 512 (find-db) vs 768 / 1024 (tuned in warmup)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for b in 512 1024 768 1024 512; do
  timeout -k 10 400 python bench.py --batch $b --warmup 12 > gpurun_out/r4f_b$b.log 2>&1 || { tail -5 gpurun_out/r4f_b$b.log; exit 1; }
  grep -h metric gpurun_out/r4f_b$b.log | cut -c1-230; grep -h "host enqueue" gpurun_out/r4f_b$b.log
  cat gpurun_out/r4f_b$b.log >> gpurun_out/r4f_all.log
done
