set -o pipefail
# depthwise statistics with the 2048-block cap and the pixels-per-block gate
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15k
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dwconv.py -m gpu > gpurun_out/${T}_pytest.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${T}_pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/${T}_pytest.log | head -20; exit 1; }
TAG=${T}_dwb0 ROUNDS=2 ARGS="--model efficientnet-b0 --batch 1024 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_DW_STATS=0" "IMGCLS_DW_STATS=1" || exit 1
TAG=${T}_dwb3 ROUNDS=2 ARGS="--model efficientnet-b3 --image-size 300 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_DW_STATS=0" "IMGCLS_DW_STATS=1" || exit 1
TAG=${T}_dwb0s ROUNDS=1 ARGS="--model efficientnet-b0 --batch 256 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_DW_STATS=0" "IMGCLS_DW_STATS=1" || exit 1
