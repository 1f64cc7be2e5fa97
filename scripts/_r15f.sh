set -o pipefail
# allocator: expandable segments vs the default caching allocator (timed-region mallocs and img/s), round 6
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15f; out=gpurun_out/${T}_alloc_ab.txt; : > $out
run() { local envs=$1; shift
  env $envs timeout -k 10 300 python bench.py "$@" > gpurun_out/${T}_run.log 2>&1 || { echo "failed: $envs $*"; tail -4 gpurun_out/${T}_run.log; return 1; }
  echo "$envs | $* | $(grep -h '^{"metric' gpurun_out/${T}_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("timed_device_malloc"), d.get("timed_device_free"))')" | tee -a $out; }
I="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8"
for r in 1 2; do
  run PYTORCH_HIP_ALLOC_CONF= $I || exit 1
  run PYTORCH_HIP_ALLOC_CONF=expandable_segments:True $I || exit 1
done
run PYTORCH_HIP_ALLOC_CONF= --batch 1024 --steps 20 --warmup 8 || exit 1
run PYTORCH_HIP_ALLOC_CONF=expandable_segments:True --batch 1024 --steps 20 --warmup 8 || exit 1
run PYTORCH_HIP_ALLOC_CONF= --model efficientnet-b3 --image-size 300 --batch 128 --steps 20 --warmup 8 || exit 1
run PYTORCH_HIP_ALLOC_CONF=expandable_segments:True --model efficientnet-b3 --image-size 300 --batch 128 --steps 20 --warmup 8 || exit 1
