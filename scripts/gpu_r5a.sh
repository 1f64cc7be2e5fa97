#!/bin/bash
# Round 3, first GPU call: (1) re-run the r4g b1536 slowdown case like for like (the 258-entry find-db that
# run loaded, 12 warmup + 30 timed steps) under a kernel trace, with allocator counters; (2) the per-GEMM
# conv roofline at the headline batch (1024).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do sleep 30; date +%s >> gpurun_out/r5a_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
timeout -k 10 500 python bench.py --batch 1536 --warmup 12 --steps 30 --tune-db tuning/r4g_find_db_258.json \
  > gpurun_out/r5a_b1536_plain.log 2>&1 || { tail -5 gpurun_out/r5a_b1536_plain.log; exit 1; }
grep -h -e metric -e allocator gpurun_out/r5a_b1536_plain.log | cut -c1-250
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5a_prof_b1536 -o hip -- \
  python3 bench.py --batch 1536 --warmup 12 --steps 30 --tune-db tuning/r4g_find_db_258.json \
  > gpurun_out/r5a_b1536_prof.log 2>&1 || { tail -5 gpurun_out/r5a_b1536_prof.log; exit 1; }
grep -h -e metric -e allocator gpurun_out/r5a_b1536_prof.log | cut -c1-250
python scripts/step_times.py gpurun_out/r5a_prof_b1536/hip_kernel_trace.csv > gpurun_out/r5a_b1536_step_times.txt
head -30 gpurun_out/r5a_b1536_step_times.txt
rm -f gpurun_out/r5a_prof_b1536/hip_kernel_trace.csv
timeout -k 10 300 python scripts/conv_roofline.py 1024 > gpurun_out/r5a_conv_roofline_b1024.txt 2>&1 || { tail -5 gpurun_out/r5a_conv_roofline_b1024.txt; exit 1; }
grep -A4 "^batch" gpurun_out/r5a_conv_roofline_b1024.txt
