set -o pipefail
# allocator traces of the timed-region mallocs, spare A/B, and the whole GPU suite on the bounds-checked library
# with MIOpen references
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r15d
timeout -k 10 300 python scripts/alloc_trace.py > gpurun_out/${T}_alloc_incep.txt 2>&1 || { tail -5 gpurun_out/${T}_alloc_incep.txt; exit 1; }
head -12 gpurun_out/${T}_alloc_incep.txt
timeout -k 10 300 python scripts/alloc_trace.py --model efficientnet-b3 --image-size 300 --batch 128 > gpurun_out/${T}_alloc_effb3.txt 2>&1 || { tail -5 gpurun_out/${T}_alloc_effb3.txt; exit 1; }
head -8 gpurun_out/${T}_alloc_effb3.txt
timeout -k 10 300 python scripts/alloc_trace.py --model resnet50 --image-size 224 --batch 1024 --steps 6 > gpurun_out/${T}_alloc_r50.txt 2>&1 || { tail -5 gpurun_out/${T}_alloc_r50.txt; exit 1; }
head -8 gpurun_out/${T}_alloc_r50.txt
TAG=${T}_spare ROUNDS=2 ARGS="--steps 20 --warmup 8" bash scripts/ab_env.sh "IMGCLS_ALLOC_SPARE=0" "IMGCLS_ALLOC_SPARE=0.25" || exit 1
IMGCLS_EXT=_C_bounds.so IMGCLS_TEST_MIOPEN=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/${T}_suite_bounds_miopen.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${T}_suite_bounds_miopen.log | tail -3
grep -E "^FAILED|out-of-bounds" gpurun_out/${T}_suite_bounds_miopen.log | head -20
exit $rc
