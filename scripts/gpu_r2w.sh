#!/bin/bash
# EfficientNet-B0 A/B: depthwise BN-backward link and fused SE kernels on/off (one box), + breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dwconv.py tests/test_hip_ops.py -k "depthwise or dw or se_gate" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2w_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/r2w_pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r2w_pytest.log | head -20; exit $rc; }
for cfg in "1 1" "0 1" "1 0" "0 0"; do
  set -- $cfg
  IMGCLS_DW_LINK=$1 IMGCLS_SE_FUSED=$2 timeout -k 10 300 python bench.py --model efficientnet-b0 --batch 256 --steps 20 --warmup 8 > gpurun_out/r2w_b0_$1$2.log 2>&1 || exit $?
  echo "link=$1 se=$2 $(tail -1 gpurun_out/r2w_b0_$1$2.log | grep -o '"value": [0-9.]*')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r2w -o hip -- python3 bench.py --model efficientnet-b0 --batch 256 --steps 3 --warmup 3 > gpurun_out/prof_r2w.log 2>&1 &&
python scripts/step_breakdown.py gpurun_out/prof_r2w/hip_kernel_trace.csv > gpurun_out/r2w_step_breakdown.txt && head -30 gpurun_out/r2w_step_breakdown.txt
