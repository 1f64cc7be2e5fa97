set -o pipefail
# BN_FIN size threshold (elements per BN output): 2M (default) vs 8M vs 32M, and off
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r15r_b4 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_MAX=8388608" || exit 1
TAG=r15r_b32 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 32 --steps 30 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" "IMGCLS_BN_FIN_MAX=8388608" "IMGCLS_BN_FIN_MAX=33554432" || exit 1
TAG=r15r_b128 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" "IMGCLS_BN_FIN_MAX=8388608" || exit 1
TAG=r15r_r50b64 ROUNDS=2 ARGS="--batch 64 --steps 30 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" "IMGCLS_BN_FIN_MAX=8388608" || exit 1
TAG=r15r_effb0 ROUNDS=1 ARGS="--model efficientnet-b0 --batch 64 --steps 30 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" "IMGCLS_BN_FIN_MAX=8388608" || exit 1
