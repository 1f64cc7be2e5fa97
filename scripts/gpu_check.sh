#!/bin/bash
# Reusable end-to-end check on one GPU box (gpurun): the whole GPU test suite, the driver's smoke step, the
# headline bench, the reference's default config (Inception-v3 @299, b4 with graph replay auto) and a
# kernel-trace step breakdown of the headline step.  TAG (env) names the outputs under gpurun_out/.
#   gpurun --timeout 1200 -- 'TAG=r7a bash scripts/gpu_check.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-check}
( while true; do sleep 30; date +%s >> gpurun_out/${T}_ticks.txt; done ) & TICK=$!
trap 'kill $TICK' EXIT
b() { local tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/${T}_$tag.log 2>&1 || { tail -5 gpurun_out/${T}_$tag.log; return 1; }
      echo "$tag $(grep -h '^{"metric' gpurun_out/${T}_$tag.log | cut -c80-150)"; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${T}_pytest_gpu.log | tail -3
case $rc in 0|1) ;; *) echo "gpu suite rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
b headline --warmup 8 --steps 20 || exit 1
b incep_b4 --model inceptionv3 --image-size 299 --batch 4 --warmup 10 --steps 60 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_prof -o hip -- \
  python3 bench.py --warmup 6 --steps 3 > gpurun_out/${T}_prof.log 2>&1 || { tail -5 gpurun_out/${T}_prof.log; exit 1; }
python scripts/step_breakdown.py gpurun_out/${T}_prof/hip_kernel_trace.csv > gpurun_out/${T}_step_breakdown.txt
python scripts/step_gaps.py gpurun_out/${T}_prof/hip_kernel_trace.csv > gpurun_out/${T}_gaps.txt
rm -f gpurun_out/${T}_prof/hip_kernel_trace.csv
head -3 gpurun_out/${T}_step_breakdown.txt
