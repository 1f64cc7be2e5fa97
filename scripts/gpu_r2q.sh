#!/bin/bash
# wgrad split-K block targets (fewer splits = less partial-tile HBM traffic beside the main stream)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for c in default 256,384,512 256 128,256; do
  if [ $c = default ]; then unset IMGCLS_WGRAD_CANDS; else export IMGCLS_WGRAD_CANDS=$c; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --tune-db none > gpurun_out/r2q_$c.log 2>&1 || exit $?
  echo "$c $(tail -1 gpurun_out/r2q_$c.log | grep -o '"value": [0-9.]*')"
done
