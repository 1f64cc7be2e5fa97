set -o pipefail
# host run-ahead (steps in flight) vs timed-region allocator events on the small-step configs (auto = 4 there)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/r15x_inflight_ab.txt; : > $out
run() { local envs=$1; shift
  env $envs timeout -k 10 300 python bench.py "$@" > gpurun_out/r15x_run.log 2>&1 || { echo "failed: $envs $*"; tail -4 gpurun_out/r15x_run.log; return 1; }
  echo "$envs | $* | $(grep -h '^{"metric' gpurun_out/r15x_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("timed_device_malloc"), d.get("timed_device_free"))')" | tee -a $out; }
for cfg in "--model resnet101 --batch 256 --steps 20 --warmup 8" "--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8" "--model inceptionv3 --image-size 299 --batch 256 --steps 20 --warmup 8" "--model efficientnet-b0 --batch 256 --steps 20 --warmup 8"; do
  for e in "IMGCLS_MAX_INFLIGHT_STEPS=-1" "IMGCLS_MAX_INFLIGHT_STEPS=2" "IMGCLS_MAX_INFLIGHT_STEPS=3"; do run "$e" $cfg || exit 1; done
done
