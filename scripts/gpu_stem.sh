#!/bin/bash
# stem kernel numerics + microbenchmark + end-to-end A/B (IMGCLS_STEM_DIRECT)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_ops.py -k "stem or pool" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_stem.log 2>&1 || { tail -40 gpurun_out/pytest_stem.log; exit 1; }
tail -1 gpurun_out/pytest_stem.log
timeout -k 10 200 python benchmarks/stem_bench.py --batch 512 > gpurun_out/stem_bench.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/stem_bench.txt
for f in 1; do
  IMGCLS_STEM_DIRECT=$f timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/abs_$f.log 2>&1 || exit $?
  echo "r50 b512 direct=$f $(tail -1 gpurun_out/abs_$f.log | cut -c80-120)"
done
