set -o pipefail
# BN_FIN apply with 4 rows of loads in flight per lane: numerics, then the size threshold again (2M / 8M / 32M)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_blocks.py -x -q --timeout 120 --timeout-method thread -k "bn_fin or inception" > gpurun_out/r15z_pytest.log 2>&1 || { tail -30 gpurun_out/r15z_pytest.log; exit 1; }
tail -1 gpurun_out/r15z_pytest.log
TAG=r15z_b4 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" || exit 1
TAG=r15z_b32 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 32 --steps 30 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" "IMGCLS_BN_FIN_MAX=8388608" "IMGCLS_BN_FIN_MAX=33554432" || exit 1
TAG=r15z_b128 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" "IMGCLS_BN_FIN_MAX=8388608" "IMGCLS_BN_FIN_MAX=33554432" || exit 1
TAG=r15z_effb0 ROUNDS=2 ARGS="--model efficientnet-b0 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" "IMGCLS_BN_FIN_MAX=8388608" || exit 1
