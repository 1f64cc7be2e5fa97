set -o pipefail
# same-box re-measure of the reference stack (torch DDP + MIOpen, bf16 autocast) against the final HIP build:
# ResNet-50 b1024 (the vs_baseline divisor), Inception-v3 b4 (the reference's own launch) and b128
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r17h_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
out=gpurun_out/r17h_refstack.txt; : > $out
run() { local tag=$1; shift
  timeout -k 10 900 python bench.py "$@" > gpurun_out/r17h_$tag.log 2>&1 || { tail -3 gpurun_out/r17h_$tag.log; return 1; }
  echo "$tag: $(grep -h '^{"metric' gpurun_out/r17h_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"]["compute"])')" | tee -a $out; }
run hip_r50 --warmup 8 --steps 20 || exit 1
run torch_r50 --compute torch --warmup 8 --steps 20 || exit 1
run hip_incep4 --model inceptionv3 --image-size 299 --batch 4 --warmup 10 --steps 60 || exit 1
run torch_incep4 --compute torch --model inceptionv3 --image-size 299 --batch 4 --warmup 10 --steps 60 || exit 1
run hip_incep128 --model inceptionv3 --image-size 299 --batch 128 --warmup 8 --steps 20 || exit 1
run torch_incep128 --compute torch --model inceptionv3 --image-size 299 --batch 128 --warmup 8 --steps 20 || exit 1
