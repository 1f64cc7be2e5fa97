set -o pipefail
# stem pool backward + BN reduce fusion (tests, A/B) and the CU-masked weight-gradient side stream (A/B), ResNet-50 b1024
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -x -q --timeout 120 --timeout-method thread -k "conv_bn_act_pool or div64" > gpurun_out/r15m_pytest.log 2>&1 || { tail -30 gpurun_out/r15m_pytest.log; exit 1; }
tail -1 gpurun_out/r15m_pytest.log
TAG=r15m_poolred ROUNDS=2 bash scripts/ab_env.sh "IMGCLS_POOL_BN_REDUCE=0" "-" || exit 1
TAG=r15m_cufrac ROUNDS=2 bash scripts/ab_env.sh "-" "IMGCLS_WGRAD_CU_FRAC=0.875" "IMGCLS_WGRAD_CU_FRAC=0.75" "IMGCLS_WGRAD_CU_FRAC=0.5" || exit 1
# allocator: do un-split large blocks reach a steady state on Inception-v3 b128? (img/s, ms, timed mallocs, frees)
out=gpurun_out/r15m_alloc_ab.txt; : > $out
I="--model inceptionv3 --image-size 299 --batch 128 --steps 20 --warmup 8"
for r in 1 2; do for conf in "" "max_split_size_mb:64"; do
  PYTORCH_HIP_ALLOC_CONF=$conf timeout -k 10 300 python bench.py $I > gpurun_out/r15m_alloc_run.log 2>&1 || { tail -4 gpurun_out/r15m_alloc_run.log; exit 1; }
  echo "PYTORCH_HIP_ALLOC_CONF=$conf | $(grep -h '^{"metric' gpurun_out/r15m_alloc_run.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("timed_device_malloc"), d.get("timed_device_free"))')" | tee -a $out
done; done
