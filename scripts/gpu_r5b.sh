#!/bin/bash
# Round 3 call b: hygiene-batch GPU tests (dense conv on MFMA kernels, weight-shadow staleness, peer timeout),
# b1536 memory diagnosis (device free memory, allocator events), conv roofline at b1024.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r5b_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_hip_ops.py -k "dense or shadow or conv_bn_act" tests/test_gpu_peer.py > gpurun_out/r5b_pytest.log 2>&1 \
  || { tail -30 gpurun_out/r5b_pytest.log; exit 1; }
tail -3 gpurun_out/r5b_pytest.log
rocm-smi --showmeminfo vram > gpurun_out/r5b_smi.txt 2>&1; head -12 gpurun_out/r5b_smi.txt
timeout -k 10 400 python bench.py --batch 1536 --warmup 12 --steps 20 > gpurun_out/r5b_b1536.log 2>&1 || { tail -5 gpurun_out/r5b_b1536.log; exit 1; }
grep -h -e metric -e memory -e allocator gpurun_out/r5b_b1536.log | cut -c1-260
timeout -k 10 300 python scripts/conv_roofline.py 1024 > gpurun_out/r5b_conv_roofline_b1024.txt 2>&1 || { tail -5 gpurun_out/r5b_conv_roofline_b1024.txt; exit 1; }
grep -A4 "^batch" gpurun_out/r5b_conv_roofline_b1024.txt
