#!/bin/bash
# Round 3 call r6e: ResNet-50 b1024 with the s2d stem weight gradient on the compute stream: two bench runs
# and a kernel-trace step breakdown (tail gap before Adam).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r6e_$tag.log 2>&1 || { tail -3 gpurun_out/r6e_$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/r6e_$tag.log | cut -c80-150)"; }
b device1 --warmup 8 --steps 20 || exit 1
b device2 --warmup 8 --steps 20 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6e_prof -o hip -- \
  python3 bench.py --warmup 6 --steps 3 > gpurun_out/r6e_prof.log 2>&1 || { tail -5 gpurun_out/r6e_prof.log; exit 1; }
python scripts/step_breakdown.py gpurun_out/r6e_prof/hip_kernel_trace.csv > gpurun_out/r6e_step_breakdown.txt
python scripts/step_gaps.py gpurun_out/r6e_prof/hip_kernel_trace.csv > gpurun_out/r6e_gaps.txt
rm -f gpurun_out/r6e_prof/hip_kernel_trace.csv
head -12 gpurun_out/r6e_step_breakdown.txt; head -14 gpurun_out/r6e_gaps.txt
