set -o pipefail
# BN_FIN with the backward counterpart (bn_reduce_bwd folded into bn_bwd_elemt): numerics, then A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_blocks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r15v_pytest.log 2>&1 || { tail -30 gpurun_out/r15v_pytest.log; exit 1; }
tail -1 gpurun_out/r15v_pytest.log
TAG=r15v_b4 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" || exit 1
TAG=r15v_b32 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 32 --steps 30 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" || exit 1
TAG=r15v_b128 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" || exit 1
TAG=r15v_r50b64 ROUNDS=2 ARGS="--batch 64 --steps 30 --warmup 8" bash scripts/ab_env.sh "IMGCLS_BN_FIN=0" "-" || exit 1
