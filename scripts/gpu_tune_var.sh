#!/bin/bash
# run-to-run variance of the per-shape tuner: N runs, each saving its choices
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/tune
ARGS=$1; R=${2:-4}
for r in $(seq 1 $R); do
  timeout -k 10 300 python bench.py $ARGS --tune-db none --tune-save gpurun_out/tune/run$r.json > gpurun_out/tune/run$r.log 2>&1 || exit $?
  echo "run$r $(tail -1 gpurun_out/tune/run$r.log | grep -o '"value": [0-9.]*')"
done
