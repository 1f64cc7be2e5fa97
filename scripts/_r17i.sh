set -o pipefail
# same-box reference stack re-measure for the remaining table rows: EfficientNet-B0 b512 and Inception-v3 b32
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r17i_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
out=gpurun_out/r17i_refstack.txt; : > $out
run() { local tag=$1; shift
  timeout -k 10 700 python bench.py "$@" > gpurun_out/r17i_$tag.log 2>&1 || { tail -3 gpurun_out/r17i_$tag.log; return 1; }
  echo "$tag: $(grep -h '^{"metric' gpurun_out/r17i_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["compute"])')" | tee -a $out; }
run hip_incep32 --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 40 || exit 1
run torch_incep32 --compute torch --model inceptionv3 --image-size 299 --batch 32 --warmup 10 --steps 40 || exit 1
run hip_effb0_512 --model efficientnet-b0 --batch 512 --warmup 8 --steps 20 || exit 1
run torch_effb0_512 --compute torch --model efficientnet-b0 --batch 512 --warmup 8 --steps 20 || exit 1
