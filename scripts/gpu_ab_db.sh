#!/bin/bash
# alternating A/B: committed find-db vs in-process tuning
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
ARGS=$1; R=${2:-3}
for r in $(seq 1 $R); do
  for db in none default; do
    if [ $db = none ]; then X="--tune-db none"; else X=""; fi
    timeout -k 10 300 python bench.py $ARGS $X > gpurun_out/ab_db.log 2>&1 || exit $?
    echo "db=$db $(tail -1 gpurun_out/ab_db.log | grep -o '"value": [0-9.]*') $(grep -o 'kernel choices from' gpurun_out/ab_db.log | head -1)"
  done
done
