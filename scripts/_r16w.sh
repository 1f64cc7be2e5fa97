set -o pipefail
# InceptionD's two 1x1 heads merged too: numerics, then Inception-v3 b4 / b128 / b256 A/B (IMGCLS_SIBLINGS=0 = per-branch everywhere)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_blocks.py tests/test_hip_ops.py -x -q --timeout 120 --timeout-method thread -k "inception" > gpurun_out/r16w_pytest.log 2>&1 || { tail -40 gpurun_out/r16w_pytest.log; exit 1; }
tail -1 gpurun_out/r16w_pytest.log
TAG=r16w_b4 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10" bash scripts/ab_env.sh "IMGCLS_SIBLINGS=0" "-" || exit 1
TAG=r16w_b256 ROUNDS=2 ARGS="--model inceptionv3 --image-size 299 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_SIBLINGS=0" "-" || exit 1
grep -h "timed at run time" gpurun_out/r16w_b256_run.log
