set -o pipefail
# find-db entries for the merged InceptionD heads: fresh tuning runs of Inception-v3 b128 / b32 / b4, each A/B'd
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r16x_incep128 RUNS=1 ARGS="--model inceptionv3 --image-size 299 --batch 128" bash scripts/retune_model.sh || exit 1
TAG=r16x_incep32 RUNS=1 ARGS="--model inceptionv3 --image-size 299 --batch 32" bash scripts/retune_model.sh || exit 1
TAG=r16x_incep4 RUNS=1 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/retune_model.sh || exit 1
