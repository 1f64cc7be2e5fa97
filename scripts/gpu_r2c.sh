#!/bin/bash
# side-stream weight gradients with a high-priority compute stream: A/B/C bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_hip_blocks.py tests/test_gpu_multirank.py tests/test_hip_ops.py -k "side_stream or two_ranks or div64" -v --timeout 300 --timeout-method thread > gpurun_out/r2c_pytest.log 2>&1; rc=$?; tail -15 gpurun_out/r2c_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
for v in "0 0" "1 0" "1 1" "0 1"; do set -- $v
IMGCLS_WGRAD_STREAM=$1 IMGCLS_HIPRIO_STEP=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r2c_bench_$1$2.$i.log 2>&1 || exit $?
echo "stream=$1 prio=$2: $(tail -1 gpurun_out/r2c_bench_$1$2.$i.log | cut -c1-140)"
done; done
