set -o pipefail
# split-K weight gradients by atomics only for layers of <= IMGCLS_WGRAD_ATOMIC_PIX output pixels
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r15p_b4 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/ab_env.sh "-" "IMGCLS_WGRAD_ATOMIC_PIX=8192" "IMGCLS_WGRAD_ATOMIC_PIX=131072" || exit 1
TAG=r15p_b32 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 32 --steps 30 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_WGRAD_ATOMIC_PIX=8192" "IMGCLS_WGRAD_ATOMIC_PIX=16384" || exit 1
TAG=r15p_b128 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_WGRAD_ATOMIC_PIX=8192" || exit 1
TAG=r15p_r50b64 ROUNDS=2 ARGS="--batch 64 --steps 30 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_WGRAD_ATOMIC_PIX=8192" "IMGCLS_WGRAD_ATOMIC_PIX=65536" || exit 1
