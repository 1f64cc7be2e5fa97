set -o pipefail
# sibling 1x1 heads as one GEMM: numerics, then Inception-v3 A/B at b4 / b32 / b128
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_blocks.py -x -q --timeout 120 --timeout-method thread -k "inception or bn_fin" > gpurun_out/r16p_pytest.log 2>&1 || { tail -40 gpurun_out/r16p_pytest.log; exit 1; }
tail -1 gpurun_out/r16p_pytest.log
TAG=r16p_b4 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/ab_env.sh "IMGCLS_SIBLINGS=0" "-" || exit 1
TAG=r16p_b32 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 32 --steps 30 --warmup 8" bash scripts/ab_env.sh "IMGCLS_SIBLINGS=0" "-" || exit 1
TAG=r16p_b128 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_SIBLINGS=0" "-" "IMGCLS_SIBLINGS_MAX=67108864" || exit 1
