set -o pipefail
# steps in flight on the small-step configs, 3 rounds: 2 vs 3 (the shipped small-step value)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r16n_incep128 ROUNDS=3 ARGS="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_MAX_INFLIGHT_STEPS=2" "-" || exit 1
TAG=r16n_incep256 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_MAX_INFLIGHT_STEPS=2" "-" || exit 1
TAG=r16n_effb0 ROUNDS=2 ARGS="--model efficientnet-b0 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_MAX_INFLIGHT_STEPS=2" "-" || exit 1
TAG=r16n_r101 ROUNDS=2 ARGS="--model resnet101 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_MAX_INFLIGHT_STEPS=2" "-" || exit 1
