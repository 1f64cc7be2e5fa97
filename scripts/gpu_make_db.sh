#!/bin/bash
# regenerate the find-db: 3 tuning runs per workload, each saving its choices (pick the fastest offline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/db
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 --tune-db none --tune-save gpurun_out/db/r50_$r.json > gpurun_out/db/r50_$r.log 2>&1 || exit $?
  echo "r50 $r $(tail -1 gpurun_out/db/r50_$r.log | grep -o '"value": [0-9.]*')"
done
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 30 --warmup 10 --tune-db none --tune-save gpurun_out/db/inc_$r.json > gpurun_out/db/inc_$r.log 2>&1 || exit $?
  echo "inc $r $(tail -1 gpurun_out/db/inc_$r.log | grep -o '"value": [0-9.]*')"
done
