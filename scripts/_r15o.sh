set -o pipefail
# split-K weight gradients by fp32 atomics into the zeroed arena slot (no workspace reduce launch) vs workspace + reduce
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r15o_b4 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/ab_env.sh "-" "IMGCLS_WGRAD_WS=0" || exit 1
TAG=r15o_b32 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 32 --steps 30 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_WGRAD_WS=0" || exit 1
TAG=r15o_b128 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_WGRAD_WS=0" || exit 1
TAG=r15o_r50 ROUNDS=1 bash scripts/ab_env.sh "-" "IMGCLS_WGRAD_WS=0" || exit 1
