set -o pipefail
# whole-step graph replay with the weight gradients forked onto the side stream inside the capture
# (IMGCLS_GRAPH_SIDE=1) against eager and the serialised capture, on this runtime (round 6)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15e; out=gpurun_out/${T}_graph_side_ab.txt; : > $out
run() { local envs=$1; shift
  env $envs timeout -k 10 300 python bench.py "$@" > gpurun_out/${T}_run.log 2>&1 || { echo "failed: $envs $*"; tail -4 gpurun_out/${T}_run.log; return 1; }
  echo "$envs | $* | $(grep -h '^{"metric' gpurun_out/${T}_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("timed_device_malloc"))')" | tee -a $out; }
I="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8"
for r in 1 2; do
  run IMGCLS_GRAPH_SIDE=0 $I --graph off || exit 1
  run IMGCLS_GRAPH_SIDE=0 $I --graph on || exit 1
  run IMGCLS_GRAPH_SIDE=1 $I --graph on || exit 1
done
run IMGCLS_GRAPH_SIDE=0 --batch 1024 --steps 20 --warmup 8 --graph off || exit 1
run IMGCLS_GRAPH_SIDE=1 --batch 1024 --steps 20 --warmup 8 --graph on || exit 1
run IMGCLS_GRAPH_SIDE=0 --model efficientnet-b0 --batch 1024 --steps 20 --warmup 8 --graph off || exit 1
run IMGCLS_GRAPH_SIDE=1 --model efficientnet-b0 --batch 1024 --steps 20 --warmup 8 --graph on || exit 1
# MIOpen's first-use kernel compile failed in the r15d suite ("Empty code object path"): where does it cache?
{ echo "HOME=$HOME USER=$(id -un) TMPDIR=$TMPDIR"; ls -ld "$HOME" "$HOME/.cache" "$HOME/.config" 2>&1; ls -la "$HOME/.cache/miopen" "$HOME/.config/miopen" 2>&1 | head; env | grep -i miopen; } > gpurun_out/${T}_miopen_env.txt 2>&1
cat gpurun_out/${T}_miopen_env.txt
timeout -k 10 300 python scripts/alloc_trace.py > gpurun_out/${T}_alloc_incep.txt 2>&1 || { tail -5 gpurun_out/${T}_alloc_incep.txt; exit 1; }
grep -A5 "device mallocs" gpurun_out/${T}_alloc_incep.txt
