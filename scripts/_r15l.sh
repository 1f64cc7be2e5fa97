set -o pipefail
# fresh find-db tuning runs for Inception-v3 b128 and EfficientNet-B0 b1024 on the current build, each A/B'd
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r15l_incep RUNS=2 ARGS="--model inceptionv3 --image-size 299 --batch 128" bash scripts/retune_model.sh || exit 1
TAG=r15l_effb0 RUNS=2 ARGS="--model efficientnet-b0 --batch 1024" bash scripts/retune_model.sh || exit 1
