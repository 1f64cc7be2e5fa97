set -o pipefail
# small-tensor BN threshold again with the preloading kernels: 2M (default) vs 8M vs 32M elements
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r17d_i256 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_MAX=8388608" "IMGCLS_BN_FIN_MAX=33554432" || exit 1
TAG=r17d_i32 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 32 --steps 30 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_MAX=8388608" || exit 1
TAG=r17d_e256 ROUNDS=2 ARGS="--model efficientnet-b0 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_MAX=8388608" || exit 1
TAG=r17d_r256 ROUNDS=2 ARGS="--batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_MAX=8388608" || exit 1
