#!/bin/bash
# fused SE MLP, depthwise BN-backward link: kernel tests, EfficientNet-B0 bench + breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dwconv.py tests/test_hip_ops.py -k "depthwise or dw or se_gate" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2v_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r2v_pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r2v_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --model efficientnet-b0 --batch 256 --steps 20 --warmup 8 > gpurun_out/r2v_b0.log 2>&1 || exit $?
grep -h "host enqueue" gpurun_out/r2v_b0.log; tail -1 gpurun_out/r2v_b0.log | grep -o '"value": [0-9.]*'
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2v -o hip -- python3 bench.py --model efficientnet-b0 --batch 256 --steps 3 --warmup 3 > gpurun_out/prof_r2v.log 2>&1 &&
python scripts/step_breakdown.py gpurun_out/prof_r2v/hip_kernel_trace.csv > gpurun_out/r2v_step_breakdown.txt && head -30 gpurun_out/r2v_step_breakdown.txt
