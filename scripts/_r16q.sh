set -o pipefail
# sibling heads merged at every size: Inception-v3 b128 / b256 / b512, 3 rounds at b128 (its run-to-run spread)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r16q_b128 ROUNDS=3 ARGS="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_SIBLINGS=0" "IMGCLS_SIBLINGS_MAX=1073741824" || exit 1
TAG=r16q_b256 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_SIBLINGS=0" "IMGCLS_SIBLINGS_MAX=1073741824" || exit 1
TAG=r16q_b512 ROUNDS=1 ARGS="--model inceptionv3 --image-size 299 --batch 512 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_SIBLINGS=0" "IMGCLS_SIBLINGS_MAX=1073741824" || exit 1
