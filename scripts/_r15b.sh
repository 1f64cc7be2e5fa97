set -o pipefail
# in-graph RCCL bucket collectives, second-BN partials centred per element, bn_res_coef_ok fallback
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15b
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -s tests/test_gpu_graph_rccl.py tests/test_gpu_rccl.py tests/test_gpu_graph.py "tests/test_hip_blocks.py::test_deferred_downsample_bn" > gpurun_out/${T}_pytest.log 2>&1; rc=$?
grep -E "passed|failed|replay ms" gpurun_out/${T}_pytest.log | tail -5
[ $rc -eq 0 ] || exit 1
IMGCLS_BN_WALK=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "tests/test_hip_blocks.py::test_deferred_downsample_bn" > gpurun_out/${T}_walk1.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_walk1.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --warmup 8 --steps 20 > gpurun_out/${T}_bench.log 2>&1 || { tail -5 gpurun_out/${T}_bench.log; exit 1; }
grep -h '^{"metric' gpurun_out/${T}_bench.log | cut -c1-200
