set -o pipefail
# Inception-v3 b4 (the reference's default launch; whole-step graph replay): where a replayed step goes
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --model inceptionv3 --image-size 299 --batch 4 --steps 50 --warmup 10 > gpurun_out/r16g_b4.log 2>&1 || { tail -5 gpurun_out/r16g_b4.log; exit 1; }
grep -h '^{"metric' gpurun_out/r16g_b4.log | cut -c1-300
MODEL=inceptionv3 RES=299 BATCH=4 bash scripts/gpu_prof_model.sh || exit 1
f=$(ls gpurun_out/prof_inceptionv3/*/hip_kernel_trace.csv gpurun_out/prof_inceptionv3/hip_kernel_trace.csv 2>/dev/null | head -1)
python scripts/step_breakdown.py "$f" > gpurun_out/r16g_incep_b4_step_breakdown.txt 2>&1 || true
python scripts/step_gaps.py "$f" > gpurun_out/r16g_incep_b4_gaps.txt 2>&1 || true
head -40 gpurun_out/r16g_incep_b4_step_breakdown.txt
