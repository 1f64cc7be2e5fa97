#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for r in 1 2; do
  for c in "256,512,1024,2048" "256,384,512,768,1024,1536,2048"; do
    IMGCLS_WGRAD_CANDS=$c timeout -k 10 300 python bench.py --steps 20 --warmup 8 --tune-db none > gpurun_out/wc.log 2>&1 || exit $?
    echo "cands=$c $(tail -1 gpurun_out/wc.log | grep -o '"value": [0-9.]*')"
  done
done
