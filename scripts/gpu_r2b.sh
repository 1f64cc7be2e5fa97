#!/bin/bash
# side-stream weight gradients: new GPU tests, then A/B bench (IMGCLS_WGRAD_STREAM=0/1, alternating)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_blocks.py tests/test_gpu_multirank.py tests/test_hip_ops.py -k "side_stream or two_ranks or div64" -x -v --timeout 300 --timeout-method thread > gpurun_out/r2b_pytest.log 2>&1; rc=$?; tail -15 gpurun_out/r2b_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
for v in 0 1; do
IMGCLS_WGRAD_STREAM=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2b_bench_s$v.$i.log 2>&1 || exit $?
echo "stream=$v: $(tail -1 gpurun_out/r2b_bench_s$v.$i.log | cut -c1-160)"
done; done
timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 --batch 128 --steps 10 --warmup 5 > gpurun_out/r2b_incep.log 2>&1 && tail -1 gpurun_out/r2b_incep.log | cut -c1-200
