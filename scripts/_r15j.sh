set -o pipefail
# stem XA (pool backward masks by the pooled output, the stem wgrad forms dY) and the depthwise-stats grid cap
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15j
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_hip_ops.py -k "pool or stem" \
  tests/test_gpu_graph.py tests/test_dwconv.py tests/test_gpu_train_e2e.py -m gpu > gpurun_out/${T}_pytest.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${T}_pytest.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" gpurun_out/${T}_pytest.log | head -20; exit 1; }
TAG=${T}_stemxa ROUNDS=2 ARGS="--batch 1024 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_STEM_XA=0" "IMGCLS_STEM_XA=1" || exit 1
TAG=${T}_dwb0 ROUNDS=2 ARGS="--model efficientnet-b0 --batch 1024 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_DW_STATS=0" "IMGCLS_DW_STATS=1" "IMGCLS_DW_STATS=1 IMGCLS_DW_STATS_GRID=2048" || exit 1
TAG=${T}_dwb3 ROUNDS=2 ARGS="--model efficientnet-b3 --image-size 300 --batch 128 --steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_DW_STATS=0" "IMGCLS_DW_STATS=1" || exit 1
