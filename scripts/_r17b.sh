set -o pipefail
# one-launch BN kernels: row blocks per 64-channel chunk (IMGCLS_BN_FIN_BLOCKS, 256 default) - the merged-head BNs ran at 1.9 TB/s at b128
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r17b_b256 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_BLOCKS=1024" "IMGCLS_BN_FIN_BLOCKS=4096" || exit 1
TAG=r17b_b4 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_BLOCKS=1024" || exit 1
TAG=r17b_b32 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 32 --steps 30 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_BLOCKS=1024" || exit 1
