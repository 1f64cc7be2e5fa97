#!/bin/bash
# Alternating on-box A/B of one switch with another fixed: gpu_ab_env2.sh VAR "FIXED=..." "bench args" [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
VAR=$1; FIX=$2; ARGS=$3; R=${4:-3}
for r in $(seq 1 $R); do
  for v in 0 1; do
    env $FIX $VAR=$v timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_env_$v.log 2>&1 || exit $?
    echo "$VAR=$v $(tail -1 gpurun_out/ab_env_$v.log | grep -o "\"value\": [0-9.]*")"
  done
done
