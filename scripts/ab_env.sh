#!/bin/bash
# Same-box interleaved A/B of bench.py under different environment settings (one process per run).
#   TAG=r5b ROUNDS=2 ARGS="--steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_XA_OUT=0" "IMGCLS_XA_OUT=1"
# Each argument is a space-separated list of VAR=value settings (use "-" for none).  One line per run in
# gpurun_out/${TAG}_ab.txt: the setting, images/sec and ms/step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-ab}; R=${ROUNDS:-2}; A=${ARGS:-"--steps 20 --warmup 8"}
out=gpurun_out/${T}_ab.txt
: > $out
for r in $(seq 1 $R); do
  for setting in "$@"; do
    envs=(); [ "$setting" != "-" ] && read -ra envs <<< "$setting"
    env "${envs[@]}" timeout -k 10 300 python bench.py $A > gpurun_out/${T}_run.log 2>&1 || { echo "run failed: $setting"; tail -5 gpurun_out/${T}_run.log; exit 1; }
    line=$(grep -h '^{"metric' gpurun_out/${T}_run.log)
    v=$(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')
    echo "round $r | $setting | $v" | tee -a $out
  done
done
