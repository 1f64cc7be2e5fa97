#!/bin/bash
# Round 3 call c: fused BN-backward (XA) correctness on the GPU, then the headline A/B (XA off / on) and a
# kernel-trace step breakdown with XA on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r5c_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hip_ops.py \
  -k "fused or conv_bn_act or dense or shadow or test_conv" > gpurun_out/r5c_pytest.log 2>&1 \
  || { tail -40 gpurun_out/r5c_pytest.log; exit 1; }
tail -3 gpurun_out/r5c_pytest.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_peer.py \
  > gpurun_out/r5c_pytest_peer.log 2>&1 || { tail -30 gpurun_out/r5c_pytest_peer.log; exit 1; }
tail -2 gpurun_out/r5c_pytest_peer.log
rocm-smi --showmeminfo vram > gpurun_out/r5c_smi.txt 2>&1; grep -i -e total -e used gpurun_out/r5c_smi.txt | head -4
IMGCLS_BN_XA=0 timeout -k 10 400 python bench.py --batch 1536 --warmup 12 --steps 10 > gpurun_out/r5c_b1536.log 2>&1 \
  || { tail -5 gpurun_out/r5c_b1536.log; exit 1; }
grep -h -e metric -e memory -e allocator gpurun_out/r5c_b1536.log | cut -c1-200
for xa in 0 1; do
  IMGCLS_BN_XA=$xa timeout -k 10 400 python bench.py --warmup 8 --steps 20 > gpurun_out/r5c_bench_xa$xa.log 2>&1 \
    || { tail -5 gpurun_out/r5c_bench_xa$xa.log; exit 1; }
  echo "xa=$xa $(grep -h metric gpurun_out/r5c_bench_xa$xa.log | cut -c80-170)"
done
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5c_prof -o hip -- \
  python3 bench.py --warmup 6 --steps 3 > gpurun_out/r5c_prof.log 2>&1 || { tail -5 gpurun_out/r5c_prof.log; exit 1; }
python scripts/step_breakdown.py gpurun_out/r5c_prof/hip_kernel_trace.csv > gpurun_out/r5c_step_breakdown.txt
python scripts/step_gaps.py gpurun_out/r5c_prof/hip_kernel_trace.csv > gpurun_out/r5c_gaps.txt
rm -f gpurun_out/r5c_prof/hip_kernel_trace.csv
head -30 gpurun_out/r5c_step_breakdown.txt; head -3 gpurun_out/r5c_gaps.txt
