set -o pipefail
# Allocator headroom (IMGCLS_ALLOC_HEADROOM, default 0.5 of the step peak, mapped after step 3): model zoo with it,
# then Inception-v3 b128 / ResNet-101 b256 with it off (same box), for the timed-region hipMalloc counts.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r17l bash scripts/bench_models.sh || exit 1
export IMGCLS_ALLOC_HEADROOM=0
TAG=r17l_off
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r17l_off_$tag.log 2>&1 || { tail -3 gpurun_out/r17l_off_$tag.log; return 1; }
      echo "off $tag $(grep -h '^{"metric' gpurun_out/r17l_off_$tag.log | grep -o '"value": [0-9.]*')"; }
b incep_b128 --model inceptionv3 --image-size 299 --batch 128 --warmup 8 --steps 20 || exit 1
b resnet101_b256 --model resnet101 --batch 256 --warmup 8 --steps 20 || exit 1
b resnet50_b1024 --batch 1024 --warmup 5 --steps 20 || exit 1
for f in gpurun_out/r17l_*.log; do echo "$f $(grep -h '^{"metric' $f | grep -o '"value": [0-9.]*\|"timed_device_malloc": [0-9]*' | tr '\n' ' ')"; done
