set -o pipefail
# Inception-v3 b128 (eager): per-queue busy time and idle gaps of one step, and the host enqueue cost
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MODEL=inceptionv3 RES=299 BATCH=128 bash scripts/gpu_prof_model.sh || exit 1
f=$(ls gpurun_out/prof_inceptionv3/hip_kernel_trace.csv 2>/dev/null | head -1)
python scripts/step_gaps.py "$f" > gpurun_out/r16i_incep_b128_gaps.txt 2>&1 || true
python scripts/step_breakdown.py "$f" > gpurun_out/r16i_incep_b128_step_breakdown.txt 2>&1 || true
rm -f "$f"
head -14 gpurun_out/r16i_incep_b128_gaps.txt; head -3 gpurun_out/r16i_incep_b128_step_breakdown.txt
grep -h "host enqueue" gpurun_out/prof_inceptionv3.log || true
