set -o pipefail
# stem pool backward + BN reduce with the BN-input loads issued up front (the first form streamed at 4.3 TB/s)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -x -q --timeout 120 --timeout-method thread -k "conv_bn_act_pool" > gpurun_out/r15t_pytest.log 2>&1 || { tail -30 gpurun_out/r15t_pytest.log; exit 1; }
tail -1 gpurun_out/r15t_pytest.log
TAG=r15t_poolred ROUNDS=3 bash scripts/ab_env.sh "IMGCLS_POOL_BN_REDUCE=0" "-" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r15t_prof -o hip -- python3 bench.py --warmup 4 --steps 2 > gpurun_out/r15t_prof.log 2>&1 || { tail -5 gpurun_out/r15t_prof.log; exit 1; }
grep -h "maxpool_bwd\|bn_bwd_reduce_u" gpurun_out/r15t_prof/hip_kernel_stats.csv | cut -c1-200
