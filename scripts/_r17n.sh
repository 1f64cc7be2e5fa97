set -o pipefail
# Save the kernel choices the tuner times at run time for the zoo configs the find-db does not cover yet
# (bench.py --tune-save), for scripts/merge_find_db.py --missing-only.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" --tune-save gpurun_out/r17n_$tag.json > gpurun_out/r17n_$tag.log 2>&1 || { tail -3 gpurun_out/r17n_$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r17n_$tag.log | grep -o '"value": [0-9.]*') $(grep -h 'timed at run time' gpurun_out/r17n_$tag.log | grep -o '[0-9]* conv, [0-9]* weight')"; }
b resnet50_b1024 --batch 1024 --warmup 5 --steps 5 || exit 1
b resnet50_b256 --batch 256 --warmup 8 --steps 5 || exit 1
b resnet50_b512 --batch 512 --warmup 8 --steps 5 || exit 1
b resnet101_b256 --model resnet101 --batch 256 --warmup 8 --steps 5 || exit 1
b incep_b256 --model inceptionv3 --image-size 299 --batch 256 --warmup 8 --steps 5 || exit 1
b incep_b512 --model inceptionv3 --image-size 299 --batch 512 --warmup 8 --steps 5 || exit 1
b effb0_b256 --model efficientnet-b0 --batch 256 --warmup 8 --steps 5 || exit 1
b effb0_b512 --model efficientnet-b0 --batch 512 --warmup 8 --steps 5 || exit 1
b effb3_b128 --model efficientnet-b3 --image-size 300 --batch 128 --warmup 8 --steps 5 || exit 1
