#!/bin/bash
# rocprofv3 kernel trace of a short bench run of MODEL (env), then per-step breakdown
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
M=${MODEL:-efficientnet-b0}; R=${RES:-224}; B=${BATCH:-256}
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$M" -o hip -- python3 "$ROOT/bench.py" --model $M --image-size $R --batch $B --steps 4 --warmup 3 > gpurun_out/prof_$M.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -1 gpurun_out/prof_$M.log | cut -c1-200
