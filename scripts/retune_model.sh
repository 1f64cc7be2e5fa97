#!/bin/bash
# Re-time every kernel choice of one bench config from scratch (bench.py --tune-db none --tune-save), RUNS times;
# keep the fastest run's find-db and A/B it against the shipped one on the same box.
#   gpurun -- 'TAG=r13m ARGS="--model efficientnet-b0" bash scripts/retune_model.sh'
# Merge a winner with: python scripts/merge_find_db.py tuning/mi355x_find_db.json gpurun_out/${TAG}_fresh_<i>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-retune}; A=${ARGS:-}; R=${RUNS:-3}
out=gpurun_out/${T}_tune.txt; : > $out
best=0; bv=0
for i in $(seq 1 $R); do
  timeout -k 10 400 python bench.py $A --warmup 5 --steps 20 --tune-db none --tune-save gpurun_out/${T}_fresh_$i.json \
    > gpurun_out/${T}_$i.log 2>&1 || { tail -5 gpurun_out/${T}_$i.log; exit 1; }
  v=$(grep -h '^{"metric' gpurun_out/${T}_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')
  echo "fresh tuning run $i: $v img/s" | tee -a $out
  if python3 -c "import sys; sys.exit(0 if $v > $bv else 1)"; then best=$i; bv=$v; fi
done
echo "best run: $best ($bv)" | tee -a $out
TAG=${T} ROUNDS=2 ARGS="$A --steps 20 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_TUNE_DB=gpurun_out/${T}_fresh_$best.json" || exit 1
cat gpurun_out/${T}_ab.txt >> $out
