set -o pipefail
# deterministic mode with fixed conv kernel choices: the same loss trajectory in separate processes, and the learning tests
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python scripts/det_check.py resnet50 96 30 32 2>&1 | grep bitwise | tee -a gpurun_out/r16e_det.txt || exit 1
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_learning.py -q -s --timeout 400 --timeout-method thread > gpurun_out/r16e_learning.log 2>&1; rc=$?
grep -E "hip loss|gaps|passed|failed" gpurun_out/r16e_learning.log | cut -c1-200
