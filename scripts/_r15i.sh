set -o pipefail
# depthwise forward with the BN statistics (DW_STATS): tests + EfficientNet A/B; layer1 conv1 fused backward A/B
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15i
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dwconv.py tests/test_models.py -m gpu > gpurun_out/${T}_pytest.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${T}_pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |Error" gpurun_out/${T}_pytest.log | head -20; exit 1; }
TAG=${T}_dwstats ROUNDS=2 ARGS="--model efficientnet-b0 --batch 1024 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_DW_STATS=0" "IMGCLS_DW_STATS=1" || exit 1
TAG=${T}_effb3 ROUNDS=1 ARGS="--model efficientnet-b3 --image-size 300 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_DW_STATS=0" "IMGCLS_DW_STATS=1" || exit 1
TAG=${T}_fbn ROUNDS=2 ARGS="--batch 1024 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_FUSED_BWD_N=0" "IMGCLS_FUSED_BWD_N=1" || exit 1
