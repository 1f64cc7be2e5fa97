set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/r7d
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r7d/$tag.log 2>&1 || { tail -3 gpurun_out/r7d/$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r7d/$tag.log | grep -o '"value": [0-9.]*')"; }
for r in 1 2; do
  b def$r --model inceptionv3 --image-size 299 --batch 256 --warmup 8 --steps 20 || exit 1
  IMGCLS_HALO=0 b nohalo$r --model inceptionv3 --image-size 299 --batch 256 --warmup 8 --steps 20 || exit 1
  IMGCLS_STEM_WGRAD_SIDE=1 b stemside$r --model inceptionv3 --image-size 299 --batch 256 --warmup 8 --steps 20 || exit 1
  IMGCLS_MAX_INFLIGHT_STEPS=4 b inflight4$r --model inceptionv3 --image-size 299 --batch 256 --warmup 8 --steps 20 || exit 1
done
