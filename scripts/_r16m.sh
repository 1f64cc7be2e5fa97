set -o pipefail
# the fp8 learning test (BASELINE config 5 compute mode)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_learning.py -q -s --timeout 300 --timeout-method thread -k fp8 > gpurun_out/r16m_fp8_learning.log 2>&1; rc=$?
grep -E "fp8:|passed|failed|Error" gpurun_out/r16m_fp8_learning.log | head; exit $rc
