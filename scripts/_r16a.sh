set -o pipefail
# BN_FIN backward form with two rows of loads in flight per lane: numerics, then A/B (IMGCLS_BN_FIN_BWD)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_blocks.py -x -q --timeout 120 --timeout-method thread -k "bn_fin" > gpurun_out/r16a_pytest.log 2>&1 || { tail -30 gpurun_out/r16a_pytest.log; exit 1; }
tail -1 gpurun_out/r16a_pytest.log
TAG=r16a_b4 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_BWD=1" || exit 1
TAG=r16a_b32 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 32 --steps 30 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_BWD=1" || exit 1
TAG=r16a_r50b64 ROUNDS=2 ARGS="--batch 64 --steps 30 --warmup 8" bash scripts/ab_env.sh "-" "IMGCLS_BN_FIN_BWD=1" || exit 1
